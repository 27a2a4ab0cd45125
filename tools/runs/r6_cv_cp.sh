#!/bin/bash
# round 6: the cross-view CP path and the suites its forward_tokens changes touch
set -o pipefail
O=gpurun_out/${OUT:-r6_cvcp}
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 900 python -u -m pytest tests/test_cp_gpu.py tests/test_crossview_gpu.py tests/test_multiview_gpu.py tests/test_dit_gpu.py tests/test_configs_net_gpu.py tests/test_tensor_abi_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
grep -E "rel-L2|CP=" $O/tests.log | tail -20
exit $rc
