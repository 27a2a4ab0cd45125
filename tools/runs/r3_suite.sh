#!/bin/bash
# round 3: the whole GPU suite and smoke() on the current tree (what the driver runs at round end)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3s
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r3s/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3s/gpu_tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r3s/gpu_tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s/smoke.log 2>&1 || { tail -20 gpurun_out/r3s/smoke.log; exit 1; }
tail -2 gpurun_out/r3s/smoke.log
