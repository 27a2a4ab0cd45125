#!/bin/bash
# round 3 (session 2): persistent cross-attention boundary isolation (lab builds: no O stores / no Q copy / no Q read /
# none of them) vs the product, then the halo conv DMA-source isolation (tools/runs/r3_conv_lab.sh)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3p
for pass in 1 2; do
  for v in product nostore nodma noqread nobound; do
    lib=""; [ $v != product ] && lib=tools/lab/libcp25_$v.so
    timeout -k 10 120 python tools/bench_xattn.py --forms 1 --rounds 2 ${lib:+--lib $lib} 2>gpurun_out/r3p/err.log | grep round | tee -a gpurun_out/r3p/xattn_probe.log | cut -c1-150 || { tail gpurun_out/r3p/err.log; exit 1; }
  done
done
bash tools/runs/r3_conv_lab.sh
