#!/bin/bash
# round 5: CP ranks' q and k|v as two GEMMs (no K|V export copy) against the fused GEMM + copy, alternating in one
# process (tools/sim_cp_rank.py --gather none --ab-split-qkv; the flag and dit.cp_split_qkv were removed with the
# rejected variant: profiles/r5/cp_sim/split_qkv_ab_rejected.log)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5cpsplit
mkdir -p $O
timeout -k 10 900 python tools/sim_cp_rank.py --cp 1 4 8 --iters 3 --gather none --ab-split-qkv > $O/sim2b_ab.log 2> $O/sim2b_ab.err || { tail -20 $O/sim2b_ab.err; exit 1; }
grep "^{" $O/sim2b_ab.log
