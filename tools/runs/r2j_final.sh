# last tree of the round: full GPU suite + smoke
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r2j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r2j/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r2j/gpu_tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r2j/gpu_tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2j/smoke.log 2>&1 || { tail -20 gpurun_out/r2j/smoke.log; exit 1; }
tail -1 gpurun_out/r2j/smoke.log
