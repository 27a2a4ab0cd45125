#!/bin/bash
# round 3 (session 2): operand ring depth of the self-attention MFMA phase (tools/lab/attn_variant.py ahead2, ahead4;
# correct results) vs the product (3 pairs ahead), zero-shift and online-max forms, same box, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3ah
for pass in 1 2 3; do
  for v in product ahead2 ahead4; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 6 ${lib:+--lib $lib} 2>gpurun_out/r3ah/err.log >> gpurun_out/r3ah/zero_ab.log || { tail gpurun_out/r3ah/err.log; exit 1; }
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --wrange 0.5,3 --iters 4 ${lib:+--lib $lib} 2>gpurun_out/r3ah/err.log >> gpurun_out/r3ah/online_ab.log || { tail gpurun_out/r3ah/err.log; exit 1; }
  done
done
for f in zero online; do echo "== $f"; python3 -c "
import json,sys
for l in open('gpurun_out/r3ah/${f}_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'], d.get('kernel',''))"; done
