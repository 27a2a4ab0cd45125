set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --num-steps 4 --no-cpu-baseline --linear-precision fp8 > $GRAFT_REPO_ROOT/gpurun_out/fprof.log 2>&1
rc=$?; grep "{" $GRAFT_REPO_ROOT/gpurun_out/fprof.log | tail -n 1 | cut -c1-300; exit $rc
