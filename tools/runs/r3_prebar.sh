#!/bin/bash
# round 3 (session 2): group B's pre-issued operand reads kept in flight across its barrier (raw barrier behind a
# counted lgkmcnt) vs the previous build (tools/lab/attn_fwd_prebar.hip), and the row-sum MFMAs first in the MFMA phase
# (tools/lab/attn_variant.py rowsum_first): attention tests, same-box A/B
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3pb
timeout -k 10 900 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attention_gpu.py tests/test_xattn_persistent_gpu.py tests/test_attn_gated_gpu.py tests/test_attn_op_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3pb/tests.log 2>&1 || { tail -30 gpurun_out/r3pb/tests.log; exit 1; }
tail -1 gpurun_out/r3pb/tests.log
A="--L 109120 --B 2 --H 16 --fused --bounded --prescaled --iters 6"
for pass in 1 2 3; do
  for v in product prebar rowsum_first; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py $A ${lib:+--lib $lib} 2>gpurun_out/r3pb/err.log >> gpurun_out/r3pb/self_ab.log || { tail gpurun_out/r3pb/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3pb/self_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"
for pass in 1 2; do
  for v in product prebar; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_xattn.py --forms 1 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3pb/err.log | grep round >> gpurun_out/r3pb/xattn_ab.log || { tail gpurun_out/r3pb/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3pb/xattn_ab.log'):
    d=json.loads(l); print(d['lib'], d['round'], d['ms'], d['tflops'])"
