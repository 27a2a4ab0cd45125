# persistent short-KV cross-attention: tests, then the DiT cross-attention shape persistent vs per-block
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/xattn_ab.log
timeout -k 10 300 python -u -m pytest tests/test_xattn_persistent_gpu.py tests/test_attention_gpu.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/xattn_tests.log 2>&1 || { tail -40 gpurun_out/xattn_tests.log; exit 1; }
tail -3 gpurun_out/xattn_tests.log
for i in 1 2; do
  CP25_XATTN_KERNEL=persist timeout -k 10 120 python tools/bench_attn.py --Lk 512 --bounded --prescaled --iters 50 >> gpurun_out/xattn_ab.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_attn.py --Lk 512 --bounded --prescaled --iters 50 >> gpurun_out/xattn_ab.log 2>&1 || exit 1
done
grep -o '"ms": [0-9.]*, "tflops": [0-9.]*' gpurun_out/xattn_ab.log
