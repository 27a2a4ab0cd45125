#!/bin/bash
# round 4, final tree: the attention tests touched by the tail symbol, then the bench script (driver command, kernel
# stats, norm-weight runs, PMC)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attn_qnorm_gpu.py tests/test_gemm_qkv_gpu.py tests/test_gemm_hnorm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
bash tools/runs/r4_bench.sh
