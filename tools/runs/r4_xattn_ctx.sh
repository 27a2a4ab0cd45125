#!/bin/bash
# round 4: the cross-attention in and out of the DiT on ONE box: the context probe, then a kernel trace of a
# one-evaluation bench (per-block cross-attention durations)
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r4xc
mkdir -p $O
timeout -k 10 200 python3 tools/xattn_context_probe.py --reps 10 > $O/probe.json 2> $O/probe.err || { tail $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o kt -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-whole-video > $O/bench.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4xc/**/kt_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
x = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if "attn_fwd_m16<1, true, 1, true" in r["Kernel_Name"]]
print("in-bench cross-attention ms:", " ".join(f"{v:.3f}" for v in x[-28:]))
print("mean of blocks 1-27 (last evaluation):", sum(x[-27:]) / 27)
PY
