#!/bin/bash
# round 3 (session 2): K tiles of group B by LDS-DMA into the padded rows (lab), same-box A/B against the product
# (tools/lab/attn_variant.py dmak) for self-attention (zero shift, online max) and the persistent cross-attention
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3dk
for pass in 1 2 3; do
  for v in product dmak dmakv; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 6 ${lib:+--lib $lib} 2>gpurun_out/r3dk/err.log >> gpurun_out/r3dk/zero_ab.log || { tail gpurun_out/r3dk/err.log; exit 1; }
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --wrange 0.5,3 --iters 4 ${lib:+--lib $lib} 2>gpurun_out/r3dk/err.log >> gpurun_out/r3dk/online_ab.log || { tail gpurun_out/r3dk/err.log; exit 1; }
    timeout -k 10 120 python tools/bench_xattn.py --forms 1 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3dk/err.log | grep round >> gpurun_out/r3dk/xattn_ab.log || { tail gpurun_out/r3dk/err.log; exit 1; }
  done
done
for f in zero online; do echo "== $f"; python3 -c "
import json
for l in open('gpurun_out/r3dk/${f}_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"; done
echo "== xattn"; python3 -c "
import json
for l in open('gpurun_out/r3dk/xattn_ab.log'):
    d=json.loads(l); print(d['lib'], d['round'], d['ms'], d['tflops'])"
