#!/bin/bash
# round 3a: the attention library's shift modes -- GPU tests, then a same-box A/B at the metric shape
# (round-2 prescaled kernel vs the zero-shift, online and weight-bound modes; unit and trained-size norm weights)
set -o pipefail
mkdir -p gpurun_out/r3a
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_attn_m16_gpu.py \
  tests/test_attention_gpu.py tests/test_attn_fp8qk_gpu.py > gpurun_out/r3a/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r3a/tests.log; exit 1; }
tail -3 gpurun_out/r3a/tests.log
for r in 1 2; do
  for cfg in "r2:--lib tools/lab/libcp25_r2.so --bounded --prescaled" "zero:--bounded --prescaled" \
             "online_unit:--normed --prescaled" "online_w3:--normed --prescaled --wrange 0.5,3" \
             "exact_q_fixed:--bounded"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python tools/bench_attn.py --fused --iters 10 $args > gpurun_out/r3a/one.json || exit 1
    echo "$name $r $(cat gpurun_out/r3a/one.json)" | tee -a gpurun_out/r3a/ab.log
  done
done
