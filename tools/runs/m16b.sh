# m16 attention with conflict-free K rows: parity tests, PMC pass, A/B vs d128 and read-ahead depth
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out/m16b
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_attn_op_gpu.py -x -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/m16b/tests.log 2>&1 || { grep -E "rel|PASS|FAIL|Error|assert" gpurun_out/m16b/tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/m16b/tests.log
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
mkdir -p gpurun_out/m16b/pmc
timeout -k 10 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/m16b/pmc -o p -- \
  python3 tools/bench_attn.py --L 109120 --B 2 --iters 1 --bounded --fused --prescaled > gpurun_out/m16b/pmc/p.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/m16b/pmc > gpurun_out/m16b/pmc/SUMMARY.json || exit 1
cat gpurun_out/m16b/pmc/SUMMARY.json
rm -f gpurun_out/m16b/ab.log
for i in 1 2; do
  CP25_ATTN_MFMA=32 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/m16b/ab.log 2>&1 || exit 1
  for lib in "" tools/lab/libcp25_ahead4.so tools/lab/libcp25_ahead2.so tools/lab/libcp25_nosched.so; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 ${lib:+--lib $lib} >> gpurun_out/m16b/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*\|"check_rel_l2": [0-9.e-]*' gpurun_out/m16b/ab.log | paste - - -
