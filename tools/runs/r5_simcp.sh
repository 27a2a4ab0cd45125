#!/bin/bash
# round 5: per-rank compute of a context-parallel rank on the final tree (tools/sim_cp_rank.py, 2B metric geometry)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5simcp
mkdir -p $O
timeout -k 10 900 python tools/sim_cp_rank.py --cp 1 2 4 8 --iters 2 > $O/sim2b.log 2> $O/sim2b.err || { tail -20 $O/sim2b.err; exit 1; }
for f in sim2b; do echo $f; grep "^{" $O/$f.log | python3 -c "
import json, sys
rows = [json.loads(l) for l in sys.stdin]
base = [r for r in rows if r['cp'] == 1][0]['forward_s']
for r in rows:
    print(r['cp'], round(r['forward_s'], 4), 'eff', round(base / r['cp'] / r['forward_s'], 4))"
done
