#!/bin/bash
# round 3e: attention tests after the range / online-trigger change, then the mode A/B
set -o pipefail
mkdir -p gpurun_out/r3e
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_attn_m16_gpu.py \
  tests/test_attention_gpu.py tests/test_fp8_gpu.py tests/test_attn_fp8qk_gpu.py \
  "tests/test_parity_depth_gpu.py::test_full_depth_2b_forward_trained_size_norm_weights" > gpurun_out/r3e/tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r3e/tests.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r3e/tests.log; exit 1; fi
for r in 1 2; do
  for cfg in "zero:--bounded --prescaled" "online_unit:--normed --prescaled" "online_w3:--normed --prescaled --wrange 0.5,3" \
             "w24_bound:--bounded --prescaled --wrange 0.5,2.3"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python tools/bench_attn.py --fused --iters 10 $args > gpurun_out/r3e/one.json || exit 1
    echo "$name $r $(cat gpurun_out/r3e/one.json)" >> gpurun_out/r3e/ab.log
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3e/ab.log"):
    n, r, j = l.split(" ", 2); d = json.loads(j); print(n, r, round(d["ms"], 2), round(d["tflops"]), d["check_rel_l2"])
PY
