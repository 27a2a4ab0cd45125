#!/bin/bash
# round 5: row sums by VALU adds of the fp32 P (vsum, lab) vs by MFMA against an all-ones row (product); metric launch
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5ab3
mkdir -p $O
B="python3 tools/bench_attn.py --fused --bounded --prescaled --qnorm"
P=cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so
for rep in 1 2 3 4; do
  for lib in $P tools/lab/libcp25_vsum.so; do
    for w in "1,1" "0.5,3"; do
      timeout -k 10 120 $B --wrange $w --iters 4 --lib $lib >> $O/ab.jsonl 2>>$O/err.log || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections, statistics
r = collections.defaultdict(list); c = {}
for l in open('gpurun_out/r5ab3/ab.jsonl'):
    d = json.loads(l); r[(d['lib'], d['wrange'])].append(d['ms']); c[d['lib']] = d['check_rel_l2']
for k, v in sorted(r.items()): print(k, [round(x, 2) for x in v], 'median', round(statistics.median(v), 2), 'check', c[k[0]])
PY
