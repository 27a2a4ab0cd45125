#!/bin/bash
# round 3 (session 2): the attention / conv builds without operand-redefining wait pins: GPU tests, then same-box A/Bs
# (self-attention vs tools/lab/attn_fwd_prenop.hip, halo conv vs tools/lab/vae_ops_prepin.hip), then the persistent
# cross-attention isolation probes
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3m
timeout -k 10 900 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attention_gpu.py tests/test_xattn_persistent_gpu.py tests/test_attn_op_gpu.py tests/test_conv_halo_gpu.py tests/test_vae_gpu.py tests/test_parity_depth_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3m/tests.log 2>&1 || { tail -30 gpurun_out/r3m/tests.log; exit 1; }
tail -1 gpurun_out/r3m/tests.log
A="--L 109120 --B 2 --H 16 --fused --bounded --prescaled --iters 6"
for pass in 1 2 3; do
  for v in product prenop; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_attn.py $A ${lib:+--lib $lib} 2>gpurun_out/r3m/err.log >> gpurun_out/r3m/self_nop_ab.log || { tail gpurun_out/r3m/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3m/self_nop_ab.log'):
    if l.startswith('{'): d=json.loads(l); print(d['lib'], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])"
for pass in 1 2; do
  for v in product convprev; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    for sh in 0 1 2; do
      CONV_LIB=$lib CONV_KINDS=halo CONV_SHAPE=$sh ROUNDS=3 timeout -k 10 120 python tools/bench_conv.py > gpurun_out/r3m/tmp.json 2>gpurun_out/r3m/err.log || { tail gpurun_out/r3m/err.log; exit 1; }
      echo "{\"pass\": $pass, \"variant\": \"$v\", \"r\": $(cat gpurun_out/r3m/tmp.json)}" | tee -a gpurun_out/r3m/conv_pin_ab.log | cut -c1-150
    done
  done
done
for pass in 1 2; do
  for v in product nostagger nodma nostore; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_xattn.py --forms 1,0 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3m/err.log | grep round >> gpurun_out/r3m/xattn_probe.log || { tail gpurun_out/r3m/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3m/xattn_probe.log'):
    d=json.loads(l); print(d['lib'], d['form'], d['round'], d['ms'], d['tflops'])"
