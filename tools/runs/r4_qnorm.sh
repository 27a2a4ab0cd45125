#!/bin/bash
# round 4: the self-attention's in-kernel q normalisation: bit-identity tests, then the metric launch A/B (the
# previous commit's attention build vs this one, without and with the in-kernel q norm)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4qn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attn_qnorm_gpu.py tests/test_attn_m16_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for rep in 1 2; do
  timeout -k 10 120 python3 tools/bench_attn.py --iters 4 --bounded --fused --prescaled --lib tools/lab/libcp25_r4head.so >> $O/ab.jsonl || exit 1
  timeout -k 10 120 python3 tools/bench_attn.py --iters 4 --bounded --fused --prescaled >> $O/ab.jsonl || exit 1
  timeout -k 10 120 python3 tools/bench_attn.py --iters 4 --bounded --fused --prescaled --qnorm >> $O/ab.jsonl || exit 1
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d = json.loads(l); print(d['lib'], 'qnorm' if d['qnorm'] else '     ', round(d['ms'], 2), round(d['tflops'], 1), d['check_rel_l2'])"
