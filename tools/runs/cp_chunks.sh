set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/bench_cp_chunks.py --cp 8 --nc 4 > gpurun_out/cpc.log 2>&1 && \
timeout -k 10 120 python tools/bench_cp_chunks.py --cp 8 --nc 2 >> gpurun_out/cpc.log 2>&1 && \
timeout -k 10 120 python tools/bench_cp_chunks.py --cp 4 --nc 4 >> gpurun_out/cpc.log 2>&1 && \
timeout -k 10 120 python tools/bench_cp_chunks.py --cp 2 --nc 4 >> gpurun_out/cpc.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_split -o run -- python tools/bench_attn.py --L 13640 --Lk 109120 --split 4 --iters 5 > gpurun_out/prof_split.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/cpc.log; find gpurun_out/prof_split -name "*stats*"; exit $rc
