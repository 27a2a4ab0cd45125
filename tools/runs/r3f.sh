#!/bin/bash
# round 3f: GEMM tests after the fp8 scale staging, fp8 / bf16 GEMM A/B, attention r2-vs-current zero mode
set -o pipefail
mkdir -p gpurun_out/r3f
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -s tests/test_gemm_gpu.py \
  > gpurun_out/r3f/tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r3f/tests.log | tail -3
if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3f/tests.log; exit 1; fi
timeout -k 10 300 python tools/bench_gemm.py --fp8 > gpurun_out/r3f/gemm_fp8.log 2>&1 || { tail gpurun_out/r3f/gemm_fp8.log; exit 1; }
cut -c1-400 gpurun_out/r3f/gemm_fp8.log
for r in 1 2; do
  for cfg in "r2:--lib tools/lab/libcp25_r2.so --bounded --prescaled" "zero:--bounded --prescaled"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python tools/bench_attn.py --fused --iters 10 $args > gpurun_out/r3f/one.json || exit 1
    echo "$name $r $(cat gpurun_out/r3f/one.json)" >> gpurun_out/r3f/ab.log
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r3f/ab.log"):
    n, r, j = l.split(" ", 2); d = json.loads(j); print(n, r, round(d["ms"], 2), round(d["tflops"]), d["check_rel_l2"])
PY
