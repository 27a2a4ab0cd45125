set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_dit_gpu.py -m gpu -x -q -s --timeout 400 --timeout-method thread -k config1 > gpurun_out/t_cfg1.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error" gpurun_out/t_cfg1.log | tail; exit $rc
