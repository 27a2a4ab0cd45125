#!/bin/bash
# round 6: the self-attention's HBM traffic, clock and MFMA busy at the bench's launch (fused q norm, prescaled, zero
# shift), three separate PMC passes (kernel-trace only), summarised for profiles/r6/bench_pmc/pmc_self.json
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-r6_pmc}
mkdir -p $O
bash tools/pmc_passes.sh $O/self python3 tools/bench_attn.py --iters 1 --bounded --fused --prescaled --qnorm || { tail -20 $O/self/p*.log; exit 1; }
python3 tools/pmc_summary.py $O/self > $O/pmc_self.json && cat $O/pmc_self.json
