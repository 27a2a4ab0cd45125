#!/bin/bash
# round 5: gemm_nt_4w isolation builds (WRONG results): DMA from L2-hot K-tiles (hot) or no DMA in the loop (nodma)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5gemm2
mkdir -p $O
for lib in cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so tools/lab/libcp25_g4w_hot.so tools/lab/libcp25_g4w_nodma.so; do
  timeout -k 10 300 python3 tools/bench_gemm.py --plain --rounds 2 --forms 0,1 --shapes qkv,mlp1 --lib $lib >> $O/plain.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 -c "
import json
for l in open('$O/plain.jsonl'):
    d = json.loads(l); print(d['lib'], d['gemm'], 'lib', [round(x,3) for x in d['hipblaslt_ms']], '8ph', [round(x,3) for x in d['own_ms_form0']], '4w', [round(x,3) for x in d['own_ms_form1']])"
