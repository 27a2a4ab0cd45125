#!/bin/bash
# round 4: config 5's action AR loop (512 frames at 480x640; bf16, fp8 block GEMMs, fp8 GEMMs + fp8 attention) and the
# 14B CP = 8 per-rank simulation (config 3) on the round-4 tree
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4e
mkdir -p $O
for cfg in "bf16 bf16" "fp8 bf16" "fp8 fp8"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_action_ar.py --linear-precision $1 --attention-precision $2 > $O/ar_$1_$2.json 2> $O/ar.err || { tail $O/ar.err; exit 1; }
  tail -n1 $O/ar_$1_$2.json
done
timeout -k 10 600 python tools/sim_cp_rank.py --cp 1 8 --iters 1 --model 14B/pre-trained > $O/sim14.log 2> $O/sim14.err || { tail -20 $O/sim14.err; exit 1; }
grep '^{' $O/sim14.log
