#!/bin/bash
# round 5: the full GPU suite and smoke() as the driver runs them, on the current tree
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5suite
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
[ $rc = 0 ] || { grep -E "FAIL|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
