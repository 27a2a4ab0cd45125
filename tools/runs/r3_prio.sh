#!/bin/bash
# round 3 (session 2): wave-priority forms of the self-attention ping-pong (tools/lab/attn_variant.py prio_b_hold,
# prio_static_b; correct results) vs the product build, same box, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3pr
A="--L 109120 --B 2 --H 16 --fused --bounded --prescaled --iters 6"
for pass in 1 2 3; do
  for v in product prio_b_hold prio_static_b; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py $A ${lib:+--lib $lib} 2>gpurun_out/r3pr/err.log >> gpurun_out/r3pr/self_ab.log || { tail gpurun_out/r3pr/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3pr/self_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"
