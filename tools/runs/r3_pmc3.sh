#!/bin/bash
# round 3 (session 2): PMC passes of the final self-attention (operand ring 2 ahead, row sums first, group B's reads
# in flight across its barrier) at the bench shape
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3pmc3
bash tools/pmc_passes.sh gpurun_out/r3pmc3/pmc_self python3 tools/bench_attn.py --iters 1 --bounded --fused --prescaled || exit 1
python3 tools/pmc_summary.py gpurun_out/r3pmc3/pmc_self > gpurun_out/r3pmc3/pmc_self.json && cat gpurun_out/r3pmc3/pmc_self.json
