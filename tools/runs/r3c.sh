#!/bin/bash
# round 3c: the tests r3b failed or did not reach (+ the fp8 GEMM), then the attention-mode A/B and the
# own-vs-library GEMM bench A/B at the metric geometry
set -o pipefail
mkdir -p gpurun_out/r3c
export PYTHONUNBUFFERED=1
timeout -k 10 1500 python -u -m pytest -v --timeout 600 --timeout-method thread -s \
  tests/test_cp_gpu.py tests/test_attn_op_gpu.py "tests/test_fp8_gpu.py::test_prescaled_attention_vs_fp32" \
  "tests/test_parity_depth_gpu.py::test_full_depth_2b_sampler" tests/test_vae_gpu.py tests/test_video_io.py \
  tests/test_gemm_gpu.py > gpurun_out/r3c/tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r3c/tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; tail -30 gpurun_out/r3c/tests.log; exit 1; fi
for r in 1 2; do
  for cfg in "r2:--lib tools/lab/libcp25_r2.so --bounded --prescaled" "zero:--bounded --prescaled" \
             "online_unit:--normed --prescaled" "online_w3:--normed --prescaled --wrange 0.5,3"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python tools/bench_attn.py --fused --iters 10 $args > gpurun_out/r3c/one.json || exit 1
    echo "$name $r $(cat gpurun_out/r3c/one.json)" >> gpurun_out/r3c/ab.log
  done
done
cat gpurun_out/r3c/ab.log | cut -c1-40,200-400
for g in own lib; do
  timeout -k 10 600 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --block-gemm $g > gpurun_out/r3c/bench_$g.json \
    2> gpurun_out/r3c/bench_$g.err || { tail -20 gpurun_out/r3c/bench_$g.err; exit 1; }
  head -c 700 gpurun_out/r3c/bench_$g.json; echo
done
