# PMC passes for both bounded self-attention kernels (2w = attn_fwd_d128, 1w = attn_fwd_1w)
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
export TMPDIR=/tmp
for kern in 1w 2w; do
  out=gpurun_out/pmc_$kern
  mkdir -p $out
  i=0
  for c in "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"; do
    i=$((i+1))
    CP25_ATTN_KERNEL=$kern timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $out -o p$i -- python3 tools/bench_attn.py --L 109120 --B 2 --iters 1 --bounded --fused --prescaled > $out/p$i.log 2>&1 || exit 1
  done
  python3 tools/pmc_dump.py $out > $out/summary.txt
  cat $out/summary.txt
done
