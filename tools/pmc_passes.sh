#!/bin/bash
# PMC passes (kernel-trace only, one counter set per run) over any benchmark command (run on the GPU box):
#   tools/pmc_passes.sh <outdir> <command ...>
#   then python tools/pmc_summary.py <outdir> --kernel <substr> --flop F --algo-bytes A > SUMMARY.json
set -e
out=$1; shift
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
  timeout -k 10 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out" -o p$i -- "$@" > "$out/p$i.log" 2>&1
done
