#!/bin/bash
# round 3 (session 2): persistent cross-attention with the spread Q copy and whole-row O stores: bit-identity tests,
# boundary isolation A/B (lab builds), then halo conv tile-width A/B (lab builds tw32 / tw64, correct results)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3q
timeout -k 10 300 python -u -m pytest tests/test_xattn_persistent_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3q/xattn_tests.log 2>&1 || { tail -30 gpurun_out/r3q/xattn_tests.log; exit 1; }
tail -1 gpurun_out/r3q/xattn_tests.log
for pass in 1 2; do
  for v in product nostore nodma nobound; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_xattn.py --forms 1,0 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3q/err.log | grep round >> gpurun_out/r3q/xattn_probe.log || { tail gpurun_out/r3q/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('gpurun_out/r3q/xattn_probe.log'):
    d=json.loads(l); print(d['lib'], d['form'], d['round'], d['ms'], d['tflops'])"
for pass in 1 2; do
  for v in product tw64 tw32; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    for sh in 0 1 2; do
      CONV_LIB=$lib CONV_KINDS=halo CONV_SHAPE=$sh ROUNDS=3 timeout -k 10 120 python tools/bench_conv.py > gpurun_out/r3q/tmp.json 2>gpurun_out/r3q/err.log || { tail gpurun_out/r3q/err.log; exit 1; }
      echo "{\"pass\": $pass, \"variant\": \"$v\", \"r\": $(cat gpurun_out/r3q/tmp.json)}" | tee -a gpurun_out/r3q/conv_tw.log | cut -c1-160
    done
  done
done
