#!/bin/bash
# round 6: every GEMM epilogue, tail-slice kernel vs the round-5 kernel, alternating on one box
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-r6_epi}
mkdir -p $O
timeout -k 10 400 python -u tools/lab/gemm_tail/ab_epi.py > $O/ab_epi.jsonl 2> $O/ab_epi.err || { tail -20 $O/ab_epi.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab_epi.jsonl'):
    d = json.loads(l); print(d['M'], d['gemm'], d['bit_identical'], d['new_min'], d['base_min'], round(d['base_over_new'], 4))"
