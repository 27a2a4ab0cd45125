set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/aprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_action_ar.py --frames 61 --linear-precision fp8 > $GRAFT_REPO_ROOT/gpurun_out/aprof.log 2>&1
rc=$?; tail -n 1 $GRAFT_REPO_ROOT/gpurun_out/aprof.log; find $GRAFT_REPO_ROOT/gpurun_out/aprof -name "*stats*"; exit $rc
