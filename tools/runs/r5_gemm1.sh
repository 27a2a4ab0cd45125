#!/bin/bash
# round 5: gemm_nt_4w bit-identity vs gemm_nt_8ph, then the plain shapes: 8ph vs 4w vs hipBLASLt at M = 218 240
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5gemm1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_4w_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/bench_gemm.py --plain --rounds 3 --forms 0,1 > $O/plain.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
python3 -c "
import json
for l in open('$O/plain.jsonl'):
    d = json.loads(l); print(d['gemm'], 'lib', [round(x,3) for x in d['hipblaslt_ms']], '8ph', [round(x,3) for x in d['own_ms_form0']], '4w', [round(x,3) for x in d['own_ms_form1']])"
