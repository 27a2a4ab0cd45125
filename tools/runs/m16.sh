# 16x16x32 attention kernel: MFMA power lab (shape lever), attention parity tests, metric-shape A/B vs the 32x32x16 kernel
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16
timeout -k 10 120 tools/lab/mfma_power 20000 > gpurun_out/m16/mfma_power.log 2>&1 || { cat gpurun_out/m16/mfma_power.log; exit 1; }
cat gpurun_out/m16/mfma_power.log
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_attn_op_gpu.py -x -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/m16/tests.log 2>&1 || { grep -E "rel|PASS|FAIL|Error|assert" gpurun_out/m16/tests.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/m16/tests.log
rm -f gpurun_out/m16/ab.log
for i in 1 2; do
  CP25_ATTN_MFMA=32 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/m16/ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/m16/ab.log 2>&1 || exit 1
done
CP25_ATTN_MFMA=32 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --iters 4 >> gpurun_out/m16/ab.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_attn.py --fused --bounded --iters 4 >> gpurun_out/m16/ab.log 2>&1 || exit 1
grep -o '"prescaled": [a-z]*\|"ms": [0-9.]*\|"check_rel_l2": [0-9.e-]*' gpurun_out/m16/ab.log | paste - - -
