#!/bin/bash
# round 4: LDS-array occupancy (SQ_LDS_IDX_ACTIVE) of the self-attention at the bench shape and of the MLP1 GEMM,
# next to MFMA busy and the clock, one counter pass each
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r4lds
mkdir -p $O
C="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/attn -o p -- python3 tools/bench_attn.py --iters 1 --bounded --fused --prescaled --qnorm > $O/attn.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/gemm -o p -- python3 tools/bench_gemm.py --plain --rounds 1 --shapes mlp1 > $O/gemm.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for tag, kern in (("attn", "attn_fwd_m16<0"), ("gemm_own", "gemm_nt_8ph"), ("gemm_lib", "Cijk")):
    f = glob.glob(f"gpurun_out/r4lds/{tag.split('_')[0]}/**/p_counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float)); span = {}
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"]); per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        span[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    d = max(per); v = per[d]; ns = span[d]
    cyc = v["GRBM_GUI_ACTIVE"] / 8
    print(tag, f"{ns/1e6:.2f} ms", f"clk {cyc/ns:.2f} GHz", {k: v[k] for k in sorted(v)},
          f"mfma_busy {v['SQ_VALU_MFMA_BUSY_CYCLES']/(1024*cyc):.3f}",
          f"lds_active/(256 cyc) {v['SQ_LDS_IDX_ACTIVE']/(256*cyc):.3f}",
          f"busy/(cyc) {v['SQ_BUSY_CYCLES']/cyc:.2f}")
PY
