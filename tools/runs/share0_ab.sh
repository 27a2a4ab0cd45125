# CFG block-0 sharing A/B on one box: whole-video bench, shared vs per-entry, interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/share0
for i in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/share0/on_$i.json 2>/dev/null || exit 1
  timeout -k 10 400 python bench.py --gpus 1 --steps 8 --warmup 2 --no-cpu-baseline --no-cfg-share > gpurun_out/share0/off_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/share0/*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value'],4), round(d['ms_per_step'],1), round(d['roofline']['avg_launch_ms'],2))"; done
