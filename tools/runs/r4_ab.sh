#!/bin/bash
# round 4: same-box interleaved A/B of attention lab builds against the product (zero shift and online max, the
# bench's fused shape). usage: LIBS="tools/lab/libcp25_x.so ..." [TESTS=...] bash tools/runs/r4_ab.sh <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4ab_$1
mkdir -p $O
P=cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
  grep -E "passed|failed|hip-ref" $O/tests.log | tail -30
fi
for pass in 1 2 3; do
  for lib in $P $LIBS; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 6 --lib $lib 2>$O/err.log >> $O/zero_ab.log || { tail $O/err.log; exit 1; }
    [ -n "$NO_ONLINE" ] || timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --wrange 0.5,3 --iters 4 --lib $lib 2>$O/err.log >> $O/online_ab.log || { tail $O/err.log; exit 1; }
  done
done
for f in zero online; do [ -f $O/${f}_ab.log ] || continue; echo "== $f"; python3 -c "
import json, collections
r = collections.defaultdict(list)
for l in open('$O/${f}_ab.log'):
    if l.startswith('{'): d = json.loads(l); r[d['lib']].append(d['ms']); chk = d['check_rel_l2']; print(d['lib'], round(d['ms'], 2), d['check_rel_l2'])
for k, v in r.items(): print('  min', k, round(min(v), 2))"; done
