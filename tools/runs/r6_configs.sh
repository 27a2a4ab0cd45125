#!/bin/bash
# round 6, final tree: config 5's action AR loop (512 frames at 480x640) in the three precisions, then configs 3 (14B,
# CP 8) and 4 (7-view multiview, CP 8) as one simulated rank beside CP 1 (tools/sim_cp_rank.py, the all-gather hidden)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_configs
mkdir -p $O
for cfg in "bf16 bf16" "fp8 bf16" "fp8 fp8"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_action_ar.py --linear-precision $1 --attention-precision $2 > $O/ar_$1_$2.json 2> $O/ar.err || { tail $O/ar.err; exit 1; }
  tail -n1 $O/ar_$1_$2.json | cut -c1-300
done
timeout -k 10 500 python tools/sim_cp_rank.py --model 14B/pre-trained --cp 1 8 --iters 2 --gather none > $O/sim14.log 2>&1 || { tail $O/sim14.log; exit 1; }
timeout -k 10 500 python tools/sim_cp_rank.py --model 2B/auto/multiview --geometry 105,27,48 --views 7 --cp 1 8 --iters 2 --gather none > $O/simmv.log 2>&1 || { tail $O/simmv.log; exit 1; }
grep -h '^{' $O/sim14.log $O/simmv.log | cut -c1-300
