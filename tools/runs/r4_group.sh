#!/bin/bash
# round 4: the GEMM's L2 tile grouping (kGroupM row tiles per group): 8 (product) vs 4 / 16 / 32, plain projections at
# M = 218 240, alternating libraries
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4gr
mkdir -p $O
for rep in 1 2; do
  for v in base g4 g16 g32; do
    timeout -k 10 120 python3 tools/bench_gemm.py --plain --rounds 2 --lib tools/lab/libcp25_$v.so >> $O/group.jsonl 2>> $O/err.log || exit 1
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/r4gr/group.jsonl"):
    d = json.loads(l)
    r[(d["gemm"], d["lib"])].append(min(d["own_ms"]))
for k, v in sorted(r.items()):
    print(k, " ".join(f"{x:.3f}" for x in v))
PY
