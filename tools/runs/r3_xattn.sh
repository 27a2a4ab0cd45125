#!/bin/bash
# round 3 (session 2): persistent cross-attention -- bit-identity tests, interleaved A/B at the DiT launch, then the
# GPU suite + smoke and the driver bench
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3x
timeout -k 10 300 python -u -m pytest tests/test_xattn_persistent_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r3x/xattn_tests.log 2>&1 || { tail -30 gpurun_out/r3x/xattn_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r3x/xattn_tests.log | tail -1
timeout -k 10 200 python -u tools/bench_xattn.py > gpurun_out/r3x/xattn_ab.log 2>&1 || { tail -20 gpurun_out/r3x/xattn_ab.log; exit 1; }
timeout -k 10 200 python -u tools/bench_xattn.py --online > gpurun_out/r3x/xattn_ab_online.log 2>&1 || { tail -20 gpurun_out/r3x/xattn_ab_online.log; exit 1; }
cat gpurun_out/r3x/xattn_ab.log gpurun_out/r3x/xattn_ab_online.log | cut -c1-200
bash tools/runs/r3_suite.sh && bash tools/runs/r3_bench.sh
