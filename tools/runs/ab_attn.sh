set -o pipefail
export PYTHONUNBUFFERED=1
VARIANTS=${VARIANTS:-"base noprio sum2n"}
: > gpurun_out/ab_attn.log
for r in 1 2 3; do
  for v in $VARIANTS; do
    timeout -k 10 60 python tools/bench_attn.py --L 109120 --iters 3 --bounded --lib tools/lab/libcp25_$v.so 2>/dev/null | grep '{' >> gpurun_out/ab_attn.log || exit 1
  done
done
python3 -c "
import json, collections
d = collections.defaultdict(list); c = {}
for l in open('gpurun_out/ab_attn.log'):
    j = json.loads(l); d[j['lib']].append(round(j['tflops'])); c[j['lib']] = j.get('check_rel_l2')
for k, v in d.items(): print(k, v, 'check', c[k])
"
