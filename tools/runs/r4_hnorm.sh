#!/bin/bash
# round 4: the cross-attention q projection with its q RMSNorm in the GEMM epilogue: bit-identity tests, timing
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4hn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_qkv_gpu.py tests/test_gemm_hnorm_gpu.py tests/test_gemm_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 120 python3 tools/bench_hnorm.py --rounds 3 > $O/bench.json || exit 1
cat $O/bench.json
