#!/bin/bash
# round 3 (session 2): (1) the self-attention MFMA phase without the operand-redefining wait pins (no s_nop pads) vs
# the previous build (tools/lab/attn_fwd_prenop.hip), interleaved processes at the bench shape; (2) the attention GPU
# tests on the new build; (3) persistent cross-attention with the staggered Q copy vs isolation builds
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3n
A="--L 109120 --B 2 --H 16 --fused --bounded --prescaled --iters 6"
for pass in 1 2 3; do
  for v in product prenop; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py $A ${lib:+--lib $lib} 2>gpurun_out/r3n/err.log | tee -a gpurun_out/r3n/self_nop_ab.log | cut -c1-60,300-420 || { tail gpurun_out/r3n/err.log; exit 1; }
  done
done
A2="--L 109120 --B 2 --H 16 --fused --bounded --prescaled --wrange 0.5,3 --iters 6"
for pass in 1 2; do
  for v in product prenop; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py $A2 ${lib:+--lib $lib} 2>gpurun_out/r3n/err.log | tee -a gpurun_out/r3n/self_nop_ab_online.log | cut -c1-60,300-420 || { tail gpurun_out/r3n/err.log; exit 1; }
  done
done
timeout -k 10 600 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attention_gpu.py tests/test_xattn_persistent_gpu.py tests/test_attn_op_gpu.py tests/test_parity_depth_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3n/attn_tests.log 2>&1 || { tail -30 gpurun_out/r3n/attn_tests.log; exit 1; }
tail -1 gpurun_out/r3n/attn_tests.log
for pass in 1 2; do
  for v in product nostagger nodma nostore; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_xattn.py --forms 1,0 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3n/err.log | grep round >> gpurun_out/r3n/xattn_probe.log || { tail gpurun_out/r3n/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3n/xattn_probe.log'):
    d=json.loads(l); print(d['lib'], d['form'], d['round'], d['ms'], d['tflops'])"
