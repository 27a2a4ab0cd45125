#!/bin/bash
# round 5: a context-parallel rank's compute with the all-gather fully hidden (tools/sim_cp_rank.py --gather none: one
# persistent buffer of real gathered K|V rows, filled in the warm-up forward), 2B at CP = 1 2 4 8 and 14B at CP = 1 8
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5simnone
mkdir -p $O
timeout -k 10 900 python tools/sim_cp_rank.py --cp 1 2 4 8 --iters 2 --gather none > $O/sim2b_none.log 2> $O/sim2b_none.err || { tail -20 $O/sim2b_none.err; exit 1; }
timeout -k 10 900 python tools/sim_cp_rank.py --model 14B/pre-trained --cp 1 8 --iters 1 --gather none > $O/sim14_none.log 2> $O/sim14_none.err || { tail -20 $O/sim14_none.err; exit 1; }
for f in sim2b_none sim14_none; do echo $f; grep "^{" $O/$f.log | python3 -c "
import json, sys
rows = [json.loads(l) for l in sys.stdin]
base = [r for r in rows if r['cp'] == 1][0]['forward_s']
for r in rows:
    print(r['cp'], round(r['forward_s'], 4), 'eff', round(base / r['cp'] / r['forward_s'], 4))"
done
