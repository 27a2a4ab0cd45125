# fp8 P.V: layout + exactness tests, then the self-attention shape bf16 prescaled vs fp8 QK vs full fp8
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/fp8pv_ab.log
timeout -k 10 300 python -u -m pytest tests/test_attn_fp8qk_gpu.py -x -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/fp8pv_tests.log 2>&1 || { tail -50 gpurun_out/fp8pv_tests.log; exit 1; }
grep -E "rel-L2|fp8 attention|passed|failed" gpurun_out/fp8pv_tests.log
for i in 1 2; do
  timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/fp8pv_ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --fp8qk --iters 4 >> gpurun_out/fp8pv_ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --fp8qk --fp8pv --iters 4 >> gpurun_out/fp8pv_ab.log 2>&1 || exit 1
done
grep -o '"fp8qk": [a-z]*\|"fp8pv": [a-z]*\|"ms": [0-9.]*' gpurun_out/fp8pv_ab.log | paste - - -
