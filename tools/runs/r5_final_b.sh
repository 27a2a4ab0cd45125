#!/bin/bash
# round 5: PMC passes of the self-attention at the bench shape (the DiT form: in-kernel q norm), and one in-bench pass
# (self-attention, MLP1 + GELU and the plain GEMM as they run inside the DiT)
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r5fb
mkdir -p $O
bash tools/pmc_passes.sh $O/pmc_self python3 tools/bench_attn.py --iters 1 --bounded --fused --prescaled --qnorm || exit 1
python3 tools/pmc_summary.py $O/pmc_self > $O/pmc_self.json && cat $O/pmc_self.json
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/inbench -o p3 -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-whole-video --trained-evals 0 > $O/inbench.log 2>&1 || exit 1
M=218240
python3 tools/pmc_summary.py $O/inbench --kernel "attn_fwd_m16<0, true, 1, false" --name "self-attention in bench" > $O/inbench_self.json
python3 tools/pmc_summary.py $O/inbench --kernel "gemm_nt_8ph<1, 2>" --name "MLP1+GELU in bench" --flop $((2*M*8192*2048)) --algo-bytes $((2*(M*2048+8192*2048+M*8192))) > $O/inbench_mlp1.json
cat $O/inbench_self.json $O/inbench_mlp1.json
# the exact-q (bounded, q rounded as the reference: one fma per score) vs the prescaled form, metric launch, same box
for rep in 1 2; do
  timeout -k 10 120 python3 tools/bench_attn.py --fused --bounded --iters 3 >> $O/exactq_vs_prescaled.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 120 python3 tools/bench_attn.py --fused --bounded --prescaled --iters 3 >> $O/exactq_vs_prescaled.jsonl 2>> $O/err.log || exit 1
done
python3 -c "
import json
for l in open('$O/exactq_vs_prescaled.jsonl'):
    d=json.loads(l); print('prescaled' if d['prescaled'] else 'exact-q', round(d['ms'],2))"
