#!/bin/bash
# round 6: the GPU suite (one process), then smoke; OUT names the gpurun_out subdirectory
set -o pipefail
O=gpurun_out/${OUT:-r6_suite}
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/tests.log | tail -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
