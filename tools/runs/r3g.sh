#!/bin/bash
# round 3g: GEMM tile-seam isolation (lab builds: no LDS staging / no global stores), then rocprofv3 kernel stats of the
# bench with the round-3 defaults (own GEMMs with fused epilogues)
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out/r3g
for r in 1 2; do
  for v in gnone nostage nostore; do
    timeout -k 10 200 python tools/bench_gemm.py --plain --rounds 1 --shapes qkv,proj,mlp1 --lib tools/lab/libcp25_$v.so \
      >> gpurun_out/r3g/seam_bf16.log 2>&1 || { tail gpurun_out/r3g/seam_bf16.log; exit 1; }
    timeout -k 10 200 python tools/bench_gemm.py --plain --fp8 --rounds 1 --shapes qkv,proj,mlp1 --lib tools/lab/libcp25_$v.so \
      >> gpurun_out/r3g/seam_fp8.log 2>&1 || { tail gpurun_out/r3g/seam_fp8.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for f in ("gpurun_out/r3g/seam_bf16.log", "gpurun_out/r3g/seam_fp8.log"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); print(d["kind"], d["lib"], d["gemm"], [round(x, 3) for x in d["own_ms"]],
                                    [round(x, 3) for x in d.get("hipblaslt_ms", d.get("scaled_mm_ms"))])
PY
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/r3g/bench_prof.json 2> gpurun_out/r3g/bench_prof.err || exit 1
python3 tools/rocpd_stats.py gpurun_out/r3g/prof/run_results.db > gpurun_out/r3g/bench_kernel_stats.csv && head -12 gpurun_out/r3g/bench_kernel_stats.csv | cut -c1-200
