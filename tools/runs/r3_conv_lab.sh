#!/bin/bash
# round 3 (session 2): halo conv DMA-source isolation (lab builds, wrong results): contiguous weight / halo DMA
# sources vs the product, two alternating passes on one box
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3c
for pass in 1 2; do
  for v in product wcontig hcontig both; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    for sh in 0 1 2; do
      CONV_LIB=$lib CONV_KINDS=halo CONV_SHAPE=$sh ROUNDS=3 timeout -k 10 120 python tools/bench_conv.py > gpurun_out/r3c/tmp.json 2>gpurun_out/r3c/err.log || { tail gpurun_out/r3c/err.log; exit 1; }
      echo "{\"pass\": $pass, \"variant\": \"$v\", \"r\": $(cat gpurun_out/r3c/tmp.json)}" | tee -a gpurun_out/r3c/conv_lab.log
    done
  done
done
