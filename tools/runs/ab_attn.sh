set -o pipefail
export PYTHONUNBUFFERED=1
VARIANTS=${VARIANTS:-"base pk wf pkwf"}
for r in 1 2 3; do
  for v in $VARIANTS; do
    timeout -k 10 60 python tools/bench_attn.py --L 109120 --iters 3 --lib tools/lab/libcp25_$v.so >> gpurun_out/ab_attn.log 2>&1 || exit 1
  done
done
grep '{' gpurun_out/ab_attn.log | python3 -c "
import sys, json, collections
d = collections.defaultdict(list); c = {}
for l in sys.stdin:
    j = json.loads(l); d[j['lib']].append(j['tflops']); c[j['lib']] = j.get('check_rel_l2')
for k, v in d.items(): print(k, ' '.join(f'{x:.0f}' for x in v), 'median', sorted(v)[len(v)//2], 'check', c[k])
"
