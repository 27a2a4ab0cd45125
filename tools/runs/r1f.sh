set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/ab_attn.log
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in "" "--bounded"; do
    timeout -k 10 60 python tools/bench_attn.py --L 109120 --iters 3 $v 2>/dev/null | grep '{' >> gpurun_out/ab_attn.log || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
