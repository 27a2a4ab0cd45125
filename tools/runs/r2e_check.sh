# re-entry check: full GPU suite + smoke on HEAD, then the fp8 options (int-P fp8 attention) at the metric geometry
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r2e
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r2e/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2e/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline --attention-precision fp8 \
  > gpurun_out/r2e/fp8_attn.json 2> gpurun_out/r2e/fp8_attn.err && \
timeout -k 10 400 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline --linear-precision fp8 --attention-precision fp8 \
  > gpurun_out/r2e/fp8_both.json 2> gpurun_out/r2e/fp8_both.err
rc=$?
grep -E "passed|failed|Error" gpurun_out/r2e/gpu_tests.log | tail -5; tail -2 gpurun_out/r2e/smoke.log
for f in fp8_attn fp8_both; do python -c "
import json
d=json.loads(open('gpurun_out/r2e/$f.json').read().strip().splitlines()[-1])
print('$f', round(d['value'],4), round(d['ms_per_step'],1), round(d['config']['seconds_per_video'],2), round(d['roofline']['achieved'],1))
" || true; done
exit $rc
