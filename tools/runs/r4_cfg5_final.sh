#!/bin/bash
# round 4, final tree: config 5's action AR loop (512 frames at 480x640) in the three precisions
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4c5
mkdir -p $O
for cfg in "bf16 bf16" "fp8 bf16" "fp8 fp8"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_action_ar.py --linear-precision $1 --attention-precision $2 > $O/ar_$1_$2.json 2> $O/ar.err || { tail $O/ar.err; exit 1; }
  tail -n1 $O/ar_$1_$2.json | cut -c1-300
done
