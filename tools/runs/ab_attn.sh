set -o pipefail
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in base st32 st16; do
    timeout -k 10 60 python tools/bench_attn.py --L 109120 --iters 3 --lib tools/lab/libcp25_$v.so >> gpurun_out/ab_attn.log 2>&1 || exit 1
  done
done
grep '{' gpurun_out/ab_attn.log | python3 -c "
import sys, json, collections
d = collections.defaultdict(list)
for l in sys.stdin:
    j = json.loads(l); d[j['lib']].append(j['tflops'])
for k, v in d.items(): print(k, ' '.join(f'{x:.0f}' for x in v), 'median', sorted(v)[len(v)//2])
"
