# config-5 fp8 options vs bf16, full metric geometry, same box
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/fp8b
timeout -k 10 500 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline --linear-precision fp8 --attention-precision fp8 \
  > gpurun_out/fp8b/fp8_both.json 2> gpurun_out/fp8b/fp8_both.err && \
timeout -k 10 500 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline --attention-precision fp8 \
  > gpurun_out/fp8b/fp8_attn.json 2> gpurun_out/fp8b/fp8_attn.err && \
timeout -k 10 500 python bench.py --gpus 1 --steps 12 --warmup 2 --no-cpu-baseline \
  > gpurun_out/fp8b/bf16.json 2> gpurun_out/fp8b/bf16.err
rc=$?
for f in fp8_both fp8_attn bf16; do python -c "
import json,sys
d=json.loads(open('gpurun_out/fp8b/$f.json').read().strip().splitlines()[-1])
print('$f', round(d['value'],4), round(d['ms_per_step'],1), round(d['config']['seconds_per_video'],2), round(d['roofline']['achieved'],1))
" || true; done
exit $rc
