#!/bin/bash
# round 3 (session 2): GPU suite + smoke, then the driver's bench command and kernel stats
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/runs/r3_suite.sh && bash tools/runs/r3_bench.sh
