#!/bin/bash
# round 5: phase anatomy of the self-attention loop (s_memtime probe build, tools/lab/build.sh probe -DCP25_ATTN_PROBE)
# beside the product's timing on the same box: zero shift (unit norm weights) and online max (weights in [0.5, 3])
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5probe
mkdir -p $O
for rep in 1 2; do
  for w in "1,1" "0.5,3"; do
    timeout -k 10 120 python3 tools/bench_attn.py --fused --bounded --prescaled --qnorm --wrange $w --iters 4 >> $O/product.jsonl 2>>$O/err.log || exit 1
    timeout -k 10 120 python3 tools/bench_attn.py --fused --bounded --prescaled --qnorm --wrange $w --iters 4 --lib tools/lab/libcp25_probe.so --probe 800 >> $O/probe.jsonl 2>>$O/err.log || exit 1
  done
done
cat $O/product.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('product', d['wrange'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"
cat $O/probe.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('probe', d['wrange'], round(d['ms'],2), json.dumps(d['probe']))"
