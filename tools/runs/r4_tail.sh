#!/bin/bash
# round 4: tail split of the last partial round of unsplit self-attention launches: tests, then same-box A/B against
# the same build with the tail disabled (tools/lab/libcp25_notail.so) at the metric shape and the CP lane shapes
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attention_gpu.py tests/test_attn_gated_gpu.py tests/test_configs_gpu.py -m gpu -x -v -s --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed|tail split" $O/tests.log | tail -3
for pass in 1 2 3; do
  for lib in tools/lab/libcp25_notail.so cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 6 --lib $lib 2>$O/err.log >> $O/metric_ab.log || { tail $O/err.log; exit 1; }
    for L in 13640 27280 54560; do
      timeout -k 10 120 python tools/bench_attn.py --B 1 --L $L --Lk 109120 --bounded --prescaled --iters 6 --lib $lib 2>$O/err.log >> $O/cp_ab.log || { tail $O/err.log; exit 1; }
    done
  done
done
for f in metric cp; do echo "== $f"; python3 -c "
import json, collections
r = collections.defaultdict(list)
for l in open('$O/${f}_ab.log'):
    if l.startswith('{'): d = json.loads(l); r[(d['Lq'], d['lib'])].append(d['ms'])
for k, v in sorted(r.items()): print(k, [round(x, 3) for x in v], 'min', round(min(v), 3))"; done
