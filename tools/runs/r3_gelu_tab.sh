#!/bin/bash
# round 3 (session 2): GELU epilogue by LDS table: GEMM / op-table tests, then MLP1 (+GELU) vs the previous build
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3t
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_op_table_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r3t/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3t/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r3t/tests.log | tail -1
grep -iE "gelu" gpurun_out/r3t/tests.log | head -5
for pass in 1 2 3; do
  for v in product gemmprev; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 200 python tools/bench_gemm.py --shapes mlp1 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3t/err.log | tee -a gpurun_out/r3t/gelu_ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], 'own', min(d['own_ms']), 'gelu fused', d['own_gelu_fused_ms'], 'lib+gelu', d['lib_plus_gelu_ms'])" || { tail gpurun_out/r3t/err.log; exit 1; }
  done
done
