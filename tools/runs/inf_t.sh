set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_inference_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/inf_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|error|assert" gpurun_out/inf_tests.log | tail -12; exit $rc
