set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_dit_gpu.py -m gpu -x -q -s --timeout 200 --timeout-method thread -k 14b > gpurun_out/t14.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error" gpurun_out/t14.log | tail; exit $rc
