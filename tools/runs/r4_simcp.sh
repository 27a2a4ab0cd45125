#!/bin/bash
# round 4: per-rank compute of the CP = 2/4/8 DiT forward on one GPU (the K/V all-gather replaced by local copies of the
# same bytes), after the attention tail split; 2B metric geometry
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4sim
mkdir -p $O
timeout -k 10 900 python tools/sim_cp_rank.py --cp 1 2 4 8 --iters 2 > $O/sim2b.log 2> $O/sim2b.err || { tail -20 $O/sim2b.err; exit 1; }
grep '^{' $O/sim2b.log
