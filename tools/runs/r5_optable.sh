#!/bin/bash
# round 5: the per-op table on the final tree, with the fp32 GEMM and affine LayerNorm rows
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5opt
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_op_table_gpu.py > gpurun_out/r5opt/tests.log 2>&1
rc=$?
grep -E "hip-ref|passed|failed" gpurun_out/r5opt/tests.log | tail -40
exit $rc
