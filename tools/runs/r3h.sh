#!/bin/bash
# round 3h: attention tests after the 16-B epilogue stores, the per-op distance table, and the cross-/self-attention
# A/B of the store tail (tools/lab/libcp25_ep8.so = the previous 8-B stores)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3h
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_attn_m16_gpu.py \
  tests/test_attention_gpu.py tests/test_op_table_gpu.py tests/test_cp_gpu.py > gpurun_out/r3h/tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r3h/tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/r3h/tests.log | head -20; exit 1; fi
grep -E "hip-ref" gpurun_out/r3h/tests.log
for r in 1 2; do
  for cfg in "ep8_x:--lib tools/lab/libcp25_ep8.so --Lk 512" "ep16_x:--Lk 512" "ep8_s:--lib tools/lab/libcp25_ep8.so --fused" "ep16_s:--fused"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python tools/bench_attn.py --bounded --prescaled --iters 20 $args > gpurun_out/r3h/one.json || exit 1
    echo "$name $r $(cat gpurun_out/r3h/one.json)" >> gpurun_out/r3h/ab.log
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3h/ab.log"):
    n, r, j = l.split(" ", 2); d = json.loads(j); print(n, r, round(d["ms"], 3), round(d["tflops"]), d["check_rel_l2"])
PY
