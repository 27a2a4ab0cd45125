#!/bin/bash
# round 4 vs round 3 on ONE box: the final round-4 tree and the round-3 final commit (1d7d643, staged under
# tools/r3_tree, not committed), the metric evaluation alternated twice (modelled per-evaluation value)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4v3
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-whole-video > $O/r4_$rep.json 2> $O/err.log || { tail $O/err.log; exit 1; }
  timeout -k 10 300 python tools/r3_tree/bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/r3_$rep.json 2> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
for rep in (1, 2):
    for t in ("r4", "r3"):
        d = json.loads(open(f"gpurun_out/r4v3/{t}_{rep}.json").read().strip().splitlines()[-1])
        print(t, rep, round(d["value"], 4), round(d["ms_per_step"], 1), round(d["roofline"].get("avg_launch_ms", 0), 2))
PY
