set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_dit_ops_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/ops_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/ops_tests.log | tail -6; exit $rc
