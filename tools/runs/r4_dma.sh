#!/bin/bash
# round 4: K/V LDS-DMA staging in the product attention: the attention GPU tests, then a same-box A/B against the
# round-3 build (tools/lab/libcp25_r3.so) for the zero-shift and online-max self-attention and the cross-attention
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4dma
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attn_gated_gpu.py tests/test_attention_gpu.py \
  tests/test_xattn_persistent_gpu.py tests/test_cp_gpu.py tests/test_dit_gpu.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for pass in 1 2 3; do
  for lib in tools/lab/libcp25_r3.so cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 6 --lib $lib 2>$O/err.log >> $O/zero_ab.log || { tail $O/err.log; exit 1; }
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --wrange 0.5,3 --iters 4 --lib $lib 2>$O/err.log >> $O/online_ab.log || { tail $O/err.log; exit 1; }
  done
done
for f in zero online; do echo "== $f"; python3 -c "
import json
for l in open('$O/${f}_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"; done
