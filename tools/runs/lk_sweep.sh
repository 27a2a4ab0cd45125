set -o pipefail
export PYTHONUNBUFFERED=1
for lk in 4160 8192 16384 32768 109120; do
  timeout -k 10 60 python tools/bench_attn.py --L 109120 --Lk $lk --iters 3 --split 1 >> gpurun_out/lk_sweep.log 2>&1 || exit 1
done
grep '{' gpurun_out/lk_sweep.log | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print(j['Lk'], round(j['ms'], 2), round(j['tflops']))
"
