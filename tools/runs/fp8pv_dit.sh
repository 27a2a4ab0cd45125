# full fp8 attention in the DiT: full-depth modes, CP=2 bit-exactness, fp8 unit tests, then the metric-geometry bench
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/fp8b
timeout -k 10 700 python -u -m pytest tests/test_parity_depth_gpu.py tests/test_cp_gpu.py tests/test_fp8_gpu.py \
  tests/test_attn_fp8qk_gpu.py -x -v -s -k "fp8 or cp2" --timeout 400 --timeout-method thread > gpurun_out/fp8pv_dit_tests.log 2>&1 \
  || { tail -40 gpurun_out/fp8pv_dit_tests.log; exit 1; }
grep -E "hip-vs-truth|CP=2|passed|failed" gpurun_out/fp8pv_dit_tests.log
timeout -k 10 500 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline --attention-precision fp8 \
  > gpurun_out/fp8b/fp8attn_full.json 2>/dev/null && \
timeout -k 10 500 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline --linear-precision fp8 --attention-precision fp8 \
  > gpurun_out/fp8b/fp8_all.json 2>/dev/null && \
timeout -k 10 500 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline \
  > gpurun_out/fp8b/bf16_b.json 2>/dev/null
rc=$?
for f in fp8attn_full fp8_all bf16_b; do python -c "
import json
d=json.loads(open('gpurun_out/fp8b/$f.json').read().strip().splitlines()[-1])
print('$f', round(d['value'],4), round(d['ms_per_step'],1), round(d['config']['seconds_per_video'],2), round(d['roofline']['avg_launch_ms'],2))
" || true; done
exit $rc
