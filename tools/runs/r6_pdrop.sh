#!/bin/bash
# round 6: fixed-shift rows shifted by min(b_row + 60, 126 - b_row) (kPDrop) -- attention / gated / qnorm / CP / DiT /
# depth / config tests, then the metric launch against the previous rule (P <= 2) and the trained-weight launch
set -o pipefail
O=gpurun_out/r6_pdrop
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 900 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attn_gated_gpu.py tests/test_attn_qnorm_gpu.py tests/test_cp_gpu.py tests/test_dit_gpu.py tests/test_parity_depth_gpu.py tests/test_configs_net_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 400 python -u tools/bench_attn.py --fused --bounded --prescaled --qnorm --iters 4 --ab 6 --ab-libs tools/lab/libcp25_prev_r6.so > $O/ab_unit.json 2> $O/ab_unit.err || { tail $O/ab_unit.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ab_unit.json')); print(d['kernel_name'], d['ab_ms']['median'], d['check_rel_l2'])"
