set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error" gpurun_out/gpu_tests_r2.log | tail -30; exit $rc
