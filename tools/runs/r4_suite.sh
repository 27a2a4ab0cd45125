#!/bin/bash
# round 4: the whole GPU suite and smoke() on the current tree (what the driver runs at round end)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/gpu_tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
