#!/bin/bash
# round 6: the CP = 8 rank simulation (gather hidden) with the GEMM tail slices (libcp25.so) and without them
# (tools/lab/gemm_tail/libcp25_base.so), alternating on one box: 2B twice each, 14B once each
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-r6_tailsim}
mkdir -p $O
BASE=tools/lab/gemm_tail/libcp25_base.so
run() {  # name, extra args
  timeout -k 10 600 python tools/sim_cp_rank.py --cp 1 8 --iters 2 --gather none $2 > $O/$1.log 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  grep "^{" $O/$1.log | python3 -c "
import json, sys
rows = [json.loads(l) for l in sys.stdin]
base = [r for r in rows if r['cp'] == 1][0]['forward_s']
print('$1', ' '.join(f\"cp{r['cp']} {r['forward_s']:.4f}s eff {base / r['cp'] / r['forward_s']:.4f}\" for r in rows))"
}
run 2b_new "" && run 2b_base "--lib $BASE" && run 2b_base2 "--lib $BASE" && run 2b_new2 "" && \
run 14b_new "--model 14B/pre-trained --iters 1" && run 14b_base "--model 14B/pre-trained --iters 1 --lib $BASE"
