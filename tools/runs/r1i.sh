set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/runs/ab_pk.sh || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1e -o run -- python bench.py > gpurun_out/bench_r1e.log 2> gpurun_out/bench_r1e.err
rc=$?; tail -1 gpurun_out/bench_r1e.log | cut -c1-600; exit $rc
