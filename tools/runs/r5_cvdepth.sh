#!/bin/bash
# round 5: the 28-block cross-view net against the fp32 truth
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5cvd
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread \
  "tests/test_parity_depth_gpu.py::test_full_depth_crossview_forward" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|hip-vs|Error" $O/tests.log | tail -10
exit $rc
