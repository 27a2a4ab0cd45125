#!/bin/bash
# round 4: the GEMM tests and the projections' timing after the per-width L2 grouping (16 row tiles for N >= 8192)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4gc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_op_table_gpu.py tests/test_gemm_qkv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 tools/bench_gemm.py --rounds 2 --shapes mlp1 > $O/mlp1.json || exit 1
cat $O/mlp1.json | cut -c1-400
