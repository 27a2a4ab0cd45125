#!/bin/bash
# round 3 (session 2): staging-load probes of the self-attention loop (tools/lab/attn_variant.py hotload, noload;
# WRONG results) vs the product, same box, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3lp
for pass in 1 2 3; do
  for v in product hotload noload; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 6 ${lib:+--lib $lib} 2>gpurun_out/r3lp/err.log >> gpurun_out/r3lp/zero_ab.log || { tail gpurun_out/r3lp/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3lp/zero_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"
