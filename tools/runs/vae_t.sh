set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/vae_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/vae_tests.log | tail -8; exit $rc
