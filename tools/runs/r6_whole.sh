#!/bin/bash
# round 6: the whole-bound fixed shift as the self-attention's default for bound products <= 63 -- attention / CP /
# DiT / depth tests, then the metric launch's kernel and time
set -o pipefail
O=gpurun_out/r6_whole
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 900 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attn_gated_gpu.py tests/test_attn_qnorm_gpu.py tests/test_cp_gpu.py tests/test_dit_gpu.py tests/test_parity_depth_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 300 python -u tools/bench_attn.py --fused --bounded --prescaled --qnorm --iters 5 > $O/attn_unit.json 2> $O/attn_unit.err || { tail $O/attn_unit.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/attn_unit.json')); print(d['kernel_name'], d['ms'], d['check_rel_l2'])"
