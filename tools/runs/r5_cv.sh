#!/bin/bash
# round 5: the cross-view multi-view net (MultiViewCrossDiT) on the device vs the oracle, and the multiview / DiT tests
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5cv
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_crossview_gpu.py tests/test_inference_gpu.py \
  tests/test_multiview_gpu.py tests/test_dit_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|rel-L2|Error" $O/tests.log | tail -30
exit $rc
