#!/bin/bash
# round 5: 14B CP = 8 rank kernel attribution (as r5_simprof.sh), and one cross-view net forward at 7 views x 8 latent
# frames of 44 x 80 (720p) on one GPU
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r5sim14
mkdir -p $O
for cp in 1 8; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p$cp -o run -- python3 tools/sim_cp_rank.py --model 14B/pre-trained --cp $cp --iters 1 > $O/sim$cp.log 2> $O/sim$cp.err || { tail -20 $O/sim$cp.err; exit 1; }
  python3 tools/rocpd_stats.py $O/p$cp/run_results.db > $O/stats$cp.csv || exit 1
  rm -rf $O/p$cp
done
timeout -k 10 500 python3 tools/sim_cp_rank.py --model 2B/auto/multiview-crossview --geometry 56,44,80 --views 7 --cp 1 --iters 2 > $O/crossview.log 2> $O/crossview.err || { tail -20 $O/crossview.err; exit 1; }
grep '^{' $O/sim1.log $O/sim8.log $O/crossview.log
