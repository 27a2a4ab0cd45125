#!/bin/bash
# round 3d: fp8 GEMM test, attention-mode A/B, GEMM A/B (bf16 + fp8), the driver-style bench own vs library GEMM,
# and the plain-command-line multi-rank rehearsal (gloo, ranks sharing the GPU)
set -o pipefail
mkdir -p gpurun_out/r3d
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -s \
  "tests/test_gemm_gpu.py::test_gemm_fp8_matches_dequantised" > gpurun_out/r3d/tests.log 2>&1
grep -E "passed|failed" gpurun_out/r3d/tests.log | tail -2
for r in 1 2; do
  for cfg in "r2:--lib tools/lab/libcp25_r2.so --bounded --prescaled" "zero:--bounded --prescaled" \
             "online_unit:--normed --prescaled" "online_w3:--normed --prescaled --wrange 0.5,3"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python tools/bench_attn.py --fused --iters 10 $args > gpurun_out/r3d/one.json || exit 1
    echo "$name $r $(cat gpurun_out/r3d/one.json)" >> gpurun_out/r3d/ab.log
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3d/ab.log"):
    n, r, j = l.split(" ", 2); d = json.loads(j); print(n, r, round(d["ms"], 2), round(d["tflops"]), d["check_rel_l2"])
PY
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/r3d/gemm_bf16.log 2>&1 || { tail gpurun_out/r3d/gemm_bf16.log; exit 1; }
timeout -k 10 300 python tools/bench_gemm.py --fp8 > gpurun_out/r3d/gemm_fp8.log 2>&1 || { tail gpurun_out/r3d/gemm_fp8.log; exit 1; }
cut -c1-300 gpurun_out/r3d/gemm_bf16.log gpurun_out/r3d/gemm_fp8.log
for g in own lib; do
  timeout -k 10 600 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --block-gemm $g > gpurun_out/r3d/bench_$g.json \
    2> gpurun_out/r3d/bench_$g.err || { tail -20 gpurun_out/r3d/bench_$g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3d/bench_$g.json'));print('$g', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['attention_kernels'])"
done
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --share-device --steps 2 --warmup 1 --no-cpu-baseline \
  --resolution 256,256 --frames 9 > gpurun_out/r3d/bench_gloo2.json 2> gpurun_out/r3d/bench_gloo2.err \
  || { tail -20 gpurun_out/r3d/bench_gloo2.err; exit 1; }
head -c 400 gpurun_out/r3d/bench_gloo2.json
