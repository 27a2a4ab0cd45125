#!/bin/bash
# round 4: staggered workgroup start on the gated-residual GEMM (x / gate loads burst at every tile seam):
# base vs stagger8 / stagger32 lab builds, the o-proj and MLP2 shapes with their LN-mod, alternating libraries
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4rs
mkdir -p $O
for rep in 1 2; do
  for v in base stg8 stg32; do
    timeout -k 10 120 python3 tools/bench_gemm.py --rounds 2 --shapes proj,mlp2 --lib tools/lab/libcp25_$v.so >> $O/res.jsonl 2>> $O/err.log || exit 1
  done
done
python3 -c "
import json
for l in open('$O/res.jsonl'):
    d = json.loads(l); print(d['gemm'], d['lib'], round(min(d['own_ms']), 3), d.get('own_residual_fused_plus_ln_mod_ms'))"
