# fp8 Q K^T attention in the DiT: full-depth precision cost, fp8 unit tests, config-5 bench A/B
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out; rm -f gpurun_out/fp8qk_short.log
timeout -k 10 600 python -u -m pytest tests/test_parity_depth_gpu.py tests/test_fp8_gpu.py tests/test_attn_fp8qk_gpu.py \
  -x -v -s --timeout 300 --timeout-method thread -k "fp8" > gpurun_out/fp8qk_dit_tests.log 2>&1 \
  || { tail -40 gpurun_out/fp8qk_dit_tests.log; exit 1; }
grep -E "hip-vs-truth|rel-L2|passed|failed" gpurun_out/fp8qk_dit_tests.log
for i in 1 2; do
  timeout -k 10 120 python tools/bench_attn.py --L 4800 --B 2 --bounded --prescaled --iters 20 >> gpurun_out/fp8qk_short.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_attn.py --L 4800 --B 2 --bounded --prescaled --fp8qk --iters 20 >> gpurun_out/fp8qk_short.log 2>&1 || exit 1
done
cut -c1-40,150-400 gpurun_out/fp8qk_short.log
