#!/bin/bash
# PMC passes over one self-attention launch at the bench shape (run on the GPU box):
#   tools/pmc_attn.sh <outdir>      then   python tools/pmc_summary.py <outdir> > profiles/rN/attn_pmc/SUMMARY.json
# Separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), kernel-trace only.
set -e
out=${1:-gpurun_out/pmc}
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p "$out"
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
)
i=0
for c in "${passes[@]}"; do
  i=$((i + 1))
  timeout -k 10 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out" -o p$i -- \
    python3 tools/bench_attn.py --L 109120 --B 2 --iters 1 --bounded --fused --prescaled > "$out/p$i.log" 2>&1
done
