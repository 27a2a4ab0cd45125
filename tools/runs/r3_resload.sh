#!/bin/bash
# round 3 (session 2): gated-residual GEMM epilogue with unserialised x / gate loads (x before the C staging), tests and
# same-box A/B vs the previous build (tools/lab/gemm_prexload.hip)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3r
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_op_table_gpu.py tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3r/tests.log 2>&1 || { tail -30 gpurun_out/r3r/tests.log; exit 1; }
tail -1 gpurun_out/r3r/tests.log
for pass in 1 2 3; do
  for v in product gemmprev; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 200 python tools/bench_gemm.py --shapes proj,mlp2 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3r/err.log | tee -a gpurun_out/r3r/res_ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['lib'], d['gemm'], 'own', round(min(d['own_ms']),3), 'own+res+lnmod', round(d['own_residual_fused_plus_ln_mod_ms'],3), 'lib+lnmod', round(d['lib_plus_ln_mod_residual_ms'],3))" || { tail gpurun_out/r3r/err.log; exit 1; }
  done
done
