# fp8 Q K^T attention: parity tests, then the DiT self-attention shape bf16-prescaled vs fp8qk, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/fp8qk_ab.log
timeout -k 10 300 python -u -m pytest tests/test_attn_fp8qk_gpu.py -x -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/fp8qk_tests.log 2>&1 || { tail -40 gpurun_out/fp8qk_tests.log; exit 1; }
grep -E "rel-L2|passed|failed" gpurun_out/fp8qk_tests.log
for i in 1 2; do
  timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/fp8qk_ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --fp8qk --iters 4 >> gpurun_out/fp8qk_ab.log 2>&1 || exit 1
done
cut -c1-40,150-400 gpurun_out/fp8qk_ab.log
