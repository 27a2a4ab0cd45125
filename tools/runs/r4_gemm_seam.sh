#!/bin/bash
# round 4: GEMM tile-seam variants (sc1 write-through C stores, staggered workgroup start) vs the same-source base,
# plain projections at M = 218 240, alternating libraries in one call (tools/lab/gemm_variant.py)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4gs
mkdir -p $O
for rep in 1 2; do
  for v in base sc1 stg8 stg32 sc1stg8; do
    timeout -k 10 120 python3 tools/bench_gemm.py --plain --rounds 3 --lib tools/lab/libcp25_$v.so >> $O/seam.log 2>> $O/err.log || exit 1
  done
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/r4gs/seam.log"):
    d = json.loads(l)
    r[(d["gemm"], d["lib"])].append(min(d["own_ms"]))
    r[(d["gemm"], "hipblaslt")].append(min(d["hipblaslt_ms"]))
for k, v in sorted(r.items()):
    print(k, " ".join(f"{x:.3f}" for x in v))
PY
