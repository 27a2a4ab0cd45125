#!/bin/bash
# round 5: the gated-residual GEMM with the next tile's DMA queued before the x / gate wait vs the previous build;
# GEMM tests, then proj and MLP2 (+ residual + LN-mod) at M = 218 240, interleaved builds; fp8 residual too
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5res
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_4w_gpu.py tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for lib in tools/lab/libcp25_gemmhead.so cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so; do
    timeout -k 10 300 python3 tools/bench_gemm.py --rounds 2 --shapes proj,mlp2 --lib $lib >> $O/res.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/res.jsonl'):
    d = json.loads(l); print(d['lib'], d['gemm'], 'plain own', [round(x,3) for x in d['own_ms']], 'res fused + ln_mod', round(d['own_residual_fused_plus_ln_mod_ms'],3), 'lib path', round(d['lib_plus_ln_mod_residual_ms'],3))"
