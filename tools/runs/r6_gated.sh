#!/bin/bash
# round 6: trained-size q/k norm weights (uniform in [0.5, 3]) at the metric shape: the default online-max attention
# vs the data-tight gated pair (--data-tight-k-bound), per-evaluation model, alternating runs on one box
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-r6_gated}
mkdir -p $O
common="--norm-weights 0.5,3 --no-whole-video --steps 6 --warmup 2 --no-cpu-baseline --trained-evals 0"
for i in 1 2; do
  for v in online gated; do
    extra=""; [ $v = gated ] && extra="--data-tight-k-bound"
    timeout -k 10 600 python bench.py $common $extra > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -20 $O/${v}_$i.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/${v}_$i.json'))
print('$v', $i, 'ms/step', round(d['ms_per_step'], 1), 'attn ms', round(d['roofline']['avg_launch_ms'], 2), d['config'].get('attention_kernels'))"
  done
done
