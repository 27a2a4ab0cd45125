#!/bin/bash
# round 5: zero-shift form, V by LDS-DMA + ring depth 3 (dmav_a3) vs the product, 6 interleaved reps, metric launch
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5ab2
mkdir -p $O
B="python3 tools/bench_attn.py --fused --bounded --prescaled --qnorm"
P=cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so
for rep in 1 2 3 4 5 6; do
  for lib in $P tools/lab/libcp25_dmav_a3.so tools/lab/libcp25_dmav.so; do
    timeout -k 10 120 $B --wrange 1,1 --iters 4 --lib $lib >> $O/ab.jsonl 2>>$O/err.log || exit 1
  done
done
python3 - <<'PY'
import json, collections, statistics
r = collections.defaultdict(list)
for l in open('gpurun_out/r5ab2/ab.jsonl'):
    d = json.loads(l); r[(d['lib'], d['wrange'])].append(d['ms'])
for k, v in sorted(r.items()): print(k, [round(x, 2) for x in v], 'min', round(min(v), 2), 'median', round(statistics.median(v), 2))
PY
