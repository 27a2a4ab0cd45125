#!/bin/bash
# round 5: same-box A/B of the self-attention (metric launch, fused shape, in-kernel q norm): the round-4 build (head),
# the product (ring depth 3 in the online form), V by LDS-DMA in the zero-shift form (dmav, dmav_a3); zero shift
# (unit weights) and online max (weights in [0.5, 3]); plus the exp isolation pair with the probe (noexp vs expdummy)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5ab1
mkdir -p $O
B="python3 tools/bench_attn.py --fused --bounded --prescaled --qnorm"
P=cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so
timeout -k 10 300 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attn_qnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for lib in tools/lab/libcp25_head.so $P tools/lab/libcp25_dmav.so tools/lab/libcp25_dmav_a3.so; do
    for w in "1,1" "0.5,3"; do
      timeout -k 10 120 $B --wrange $w --iters 4 --lib $lib >> $O/ab.jsonl 2>>$O/err.log || exit 1
    done
  done
done
for rep in 1 2; do
  for lib in p_noexp p_expdummy; do
    timeout -k 10 120 $B --wrange 1,1 --iters 4 --lib tools/lab/libcp25_$lib.so --probe 800 >> $O/probe.jsonl 2>>$O/err.log || exit 1
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open('gpurun_out/r5ab1/ab.jsonl'):
    d = json.loads(l); r[(d['lib'], d['wrange'])].append(d['ms'])
for k, v in sorted(r.items()): print(k, [round(x, 2) for x in v], 'min', round(min(v), 2), d['check_rel_l2'])
for l in open('gpurun_out/r5ab1/probe.jsonl'):
    d = json.loads(l); p = d['probe']; print(d['lib'], round(d['ms'], 2), p['period'], p['clock_ghz'])
PY
