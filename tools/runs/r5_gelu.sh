#!/bin/bash
# round 5: the GELU epilogue after the read-back (under the next tile's DMA) vs the round-4 build (in the C staging):
# GEMM tests, then MLP1 + GELU fused at M = 218 240, interleaved builds
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5gelu
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_4w_gpu.py tests/test_gemm_qkv_gpu.py tests/test_gemm_hnorm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for lib in tools/lab/libcp25_gemmhead.so cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so; do
    timeout -k 10 300 python3 tools/bench_gemm.py --rounds 2 --shapes mlp1 --lib $lib >> $O/mlp1.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/mlp1.jsonl'):
    d = json.loads(l); print(d['lib'], 'plain own', [round(x,3) for x in d['own_ms']], 'lib', [round(x,3) for x in d['hipblaslt_ms']], 'gelu fused', round(d['own_gelu_fused_ms'],3), 'lib+gelu', round(d['lib_plus_gelu_ms'],3))"
