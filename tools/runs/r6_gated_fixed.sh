#!/bin/bash
# round 6: the gated pair's first launch on the fixed shift (measured key bound) -- gated / qnorm / CP tests, then the
# in-DiT ABBA against the online max with trained-size norm weights
set -o pipefail
O=gpurun_out/r6_gfix
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 900 python -u -m pytest tests/test_attn_gated_gpu.py tests/test_attn_qnorm_gpu.py tests/test_attn_m16_gpu.py tests/test_cp_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 700 python -u tools/ab_whole_shift.py --pairs 6 --trained > $O/ab_trained.json 2> $O/ab_trained.err || { tail $O/ab_trained.err; exit 1; }
cat $O/ab_trained.json
