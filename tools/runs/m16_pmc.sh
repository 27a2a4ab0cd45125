# 16x16x32 vs 32x32x16 attention: one SQ + GRBM PMC pass each (clock, MFMA busy, wave split), then read-ahead A/B
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for v in 32 16; do
  mkdir -p gpurun_out/m16pmc/$v
  CP25_ATTN_MFMA=$v timeout -k 10 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/m16pmc/$v -o p -- \
    python3 tools/bench_attn.py --L 109120 --B 2 --iters 1 --bounded --fused --prescaled > gpurun_out/m16pmc/$v/p.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/m16pmc/$v > gpurun_out/m16pmc/$v/SUMMARY.json || exit 1
  cat gpurun_out/m16pmc/$v/SUMMARY.json
done
rm -f gpurun_out/m16pmc/ab.log
for i in 1 2; do
  for lib in "" tools/lab/libcp25_ahead4.so tools/lab/libcp25_ahead6.so; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 ${lib:+--lib $lib} >> gpurun_out/m16pmc/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*' gpurun_out/m16pmc/ab.log | paste - -
