#!/bin/bash
# round 3b: the whole GPU suite on the round-3 tree (shift modes, own GEMM default, new config tests), then the
# attention-mode A/B and an own-vs-library GEMM bench A/B at the metric geometry
set -o pipefail
mkdir -p gpurun_out/r3b
export PYTHONUNBUFFERED=1
timeout -k 10 2400 python -u -m pytest -v --maxfail=15 --timeout 600 --timeout-method thread -m gpu -s tests/ \
  > gpurun_out/r3b/tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r3b/tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; tail -30 gpurun_out/r3b/tests.log; exit 1; fi
for r in 1 2; do
  for cfg in "r2:--lib tools/lab/libcp25_r2.so --bounded --prescaled" "zero:--bounded --prescaled" \
             "online_unit:--normed --prescaled" "online_w3:--normed --prescaled --wrange 0.5,3"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 180 python tools/bench_attn.py --fused --iters 10 $args > gpurun_out/r3b/one.json || exit 1
    echo "$name $r $(cat gpurun_out/r3b/one.json)" | tee -a gpurun_out/r3b/ab.log
  done
done
for g in own lib; do
  timeout -k 10 600 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --block-gemm $g > gpurun_out/r3b/bench_$g.json \
    2> gpurun_out/r3b/bench_$g.err || { tail -20 gpurun_out/r3b/bench_$g.err; exit 1; }
  tail -c 600 gpurun_out/r3b/bench_$g.json
done
