set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error" gpurun_out/gpu_tests.log | tail -20; tail -2 gpurun_out/smoke.log; exit $rc
