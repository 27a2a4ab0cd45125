#!/bin/bash
# round 3j: halo conv with 8 waves (two per SIMD) vs 4: bit-identity tests and the decoder-shape A/B
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3j
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -s tests/test_conv_halo_gpu.py \
  > gpurun_out/r3j/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3j/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r3j/tests.log | tail -1
CONV_KINDS=halo,halo8,tap ROUNDS=3 timeout -k 10 300 python tools/bench_conv.py > gpurun_out/r3j/bench_conv.log 2>&1 || { tail gpurun_out/r3j/bench_conv.log; exit 1; }
cat gpurun_out/r3j/bench_conv.log
