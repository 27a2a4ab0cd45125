#!/bin/bash
# round 5: kernel-time attribution of a CP = 8 rank vs CP = 1 (tools/sim_cp_rank.py under rocprofv3 --stats)
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r5simprof
mkdir -p $O
for cp in 1 8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p$cp -o run -- python3 tools/sim_cp_rank.py --cp $cp --iters 1 > $O/sim$cp.log 2> $O/sim$cp.err || { tail -20 $O/sim$cp.err; exit 1; }
  python3 tools/rocpd_stats.py $O/p$cp/run_results.db > $O/stats$cp.csv || exit 1
  rm -rf $O/p$cp
done
ls $O
