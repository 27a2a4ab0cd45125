#!/bin/bash
# PMC passes over the VAE's 96-channel full-resolution 3x3x3 conv (704 x 1280, 4 output frames), halo kernel and
# per-tap kernel in the same process (run on the GPU box):
#   tools/pmc_conv.sh <outdir>   then   python tools/pmc_conv_summary.py <outdir> > profiles/rN/conv_pmc/SUMMARY.json
set -e
out=${1:-gpurun_out/pmc_conv}
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p "$out"
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
)
i=0
for c in "${passes[@]}"; do
  i=$((i + 1))
  CONV_SHAPE=0 ROUNDS=1 timeout -k 10 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out" -o p$i -- \
    python3 tools/bench_conv.py > "$out/p$i.log" 2>&1
done
