#!/bin/bash
# round 3 (session 2): the two pending A/Bs in one box: attention barrier / row-sum order, GEMM residual loads
set -o pipefail
bash tools/runs/r3_resload.sh && bash tools/runs/r3_prebar.sh
