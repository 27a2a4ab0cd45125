# full GPU suite + smoke (the driver's round-end checks)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/gpu_tests_r2.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r2.log 2>&1
rc=$?; tail -3 gpurun_out/smoke_r2.log; exit $rc
