set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/sim_cp_rank.py --cp 1 2 4 8 > gpurun_out/sim_cp.log 2>&1 && \
timeout -k 10 300 python tools/sim_cp_rank.py --cp 1 --force-lanes >> gpurun_out/sim_cp.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sim_cp.log | grep '{'; tail -1 gpurun_out/bench.log | cut -c1-700; exit $rc
