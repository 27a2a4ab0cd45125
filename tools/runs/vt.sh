# V^T tile layout for the 16x16x32 attention: parity tests, then bench A/B (CP25_ATTN_VT=0 vs 1) at the metric geometry
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/vt
timeout -k 10 500 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_cp_gpu.py tests/test_attn_op_gpu.py tests/test_dit_gpu.py tests/test_parity_depth_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/vt/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/vt/tests.log | tail -30; exit 1; }
grep -E "passed|failed|hip-vs-truth" gpurun_out/vt/tests.log | tail -6
for i in 1 2; do
  for m in 0 1; do
    CP25_ATTN_VT=$m timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/vt/vt$m.$i.json 2> gpurun_out/vt/vt$m.$i.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/vt/vt$m.$i.json').read().strip().splitlines()[-1]); print('vt=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
