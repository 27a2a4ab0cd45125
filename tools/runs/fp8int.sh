# integer-byte fp8 P vs exp2 fp8 P: tests, then the self-attention shape A/B
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/fp8int_ab.log
timeout -k 10 300 python -u -m pytest tests/test_attn_fp8qk_gpu.py -x -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/fp8int_tests.log 2>&1 || { tail -50 gpurun_out/fp8int_tests.log; exit 1; }
grep -E "fp8 attention|passed|failed" gpurun_out/fp8int_tests.log
for i in 1 2; do
  CP25_F8_EXP=exact timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --fp8qk --fp8pv --iters 4 >> gpurun_out/fp8int_ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --fp8qk --fp8pv --iters 4 >> gpurun_out/fp8int_ab.log 2>&1 || exit 1
done
grep -o '"ms": [0-9.]*' gpurun_out/fp8int_ab.log
