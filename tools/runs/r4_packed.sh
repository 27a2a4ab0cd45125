#!/bin/bash
# round 4: the packed-f32 q normalisation prologue: attention tests, then the metric launch A/B against the
# previous build (with and without the in-kernel q normalisation)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4pk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attn_qnorm_gpu.py tests/test_attn_m16_gpu.py tests/test_attn_gated_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for q in "" "--qnorm"; do
    timeout -k 10 120 python3 tools/bench_attn.py --iters 4 --bounded --fused --prescaled $q --lib tools/lab/libcp25_prepk.so >> $O/ab.jsonl || exit 1
    timeout -k 10 120 python3 tools/bench_attn.py --iters 4 --bounded --fused --prescaled $q >> $O/ab.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d = json.loads(l); print(d['lib'], 'qnorm' if d['qnorm'] else '     ', round(d['ms'], 2), round(d['tflops'], 1), d['check_rel_l2'])"
