#!/bin/bash
# round 6: long-key launches with bound products up to 110 on the fixed shift -- attention / gated / qnorm / CP / DiT /
# depth tests, then the launch-level A/B against the previous routing (zero shift for 63 < b <= 96) at norm weights in
# [0.5, 2] (bound product ~68) and the unit-weight case
set -o pipefail
O=gpurun_out/r6_f110
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 900 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attn_gated_gpu.py tests/test_attn_qnorm_gpu.py tests/test_cp_gpu.py tests/test_dit_gpu.py tests/test_parity_depth_gpu.py tests/test_configs_net_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 400 python -u tools/bench_attn.py --fused --bounded --prescaled --qnorm --wrange 0.5,2 --iters 4 --ab 6 --ab-libs tools/lab/libcp25_prev_r6.so > $O/ab_w2.json 2> $O/ab_w2.err || { tail $O/ab_w2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ab_w2.json')); print(d['kernel_name'], d['ab_ms']['median'], d['ab_ms']['bit_identical'])"
