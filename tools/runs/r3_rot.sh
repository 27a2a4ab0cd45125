#!/bin/bash
# round 3 (session 2): group A Q K^T first with pre-issued reads: attention tests, same-box A/B against the previous build
# (tools/lab/attn_variant.py prerot) for self-attention (zero shift, online max) and the persistent cross-attention
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3rot
timeout -k 10 900 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attention_gpu.py tests/test_xattn_persistent_gpu.py tests/test_attn_gated_gpu.py tests/test_attn_op_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3rot/tests.log 2>&1 || { tail -30 gpurun_out/r3rot/tests.log; exit 1; }
tail -1 gpurun_out/r3rot/tests.log
for pass in 1 2 3; do
  for v in product prerot; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 6 ${lib:+--lib $lib} 2>gpurun_out/r3rot/err.log >> gpurun_out/r3rot/zero_ab.log || { tail gpurun_out/r3rot/err.log; exit 1; }
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --wrange 0.5,3 --iters 4 ${lib:+--lib $lib} 2>gpurun_out/r3rot/err.log >> gpurun_out/r3rot/online_ab.log || { tail gpurun_out/r3rot/err.log; exit 1; }
    timeout -k 10 120 python tools/bench_xattn.py --forms 1 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3rot/err.log | grep round >> gpurun_out/r3rot/xattn_ab.log || { tail gpurun_out/r3rot/err.log; exit 1; }
  done
done
for f in zero online; do echo "== $f"; python3 -c "
import json
for l in open('gpurun_out/r3rot/${f}_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"; done
echo "== xattn"; python3 -c "
import json
for l in open('gpurun_out/r3rot/xattn_ab.log'):
    d=json.loads(l); print(d['lib'], d['round'], d['ms'], d['tflops'])"
