"""Summarise tools/pmc_conv.sh: per conv kernel (last dispatch of each), HBM bytes (FETCH_SIZE x2 on gfx950 per
MI355X_MICROARCH.md §HBM, WRITE_SIZE), MFMA busy, clock, TFLOP/s, LDS instructions and bank conflicts.
usage: python tools/pmc_conv_summary.py gpurun_out/pmc_conv
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {"conv3x3_halo_kernel": "halo (LDS halo tile, round 2)", "conv_igemm_kernel": "per-tap implicit GEMM (round 1)"}
H, W, C, TOUT = 704, 1280, 96, 4
FLOP = 2.0 * 27 * C * C * H * W * TOUT
ALGO = (TOUT + 2) * H * W * C * 2 + TOUT * H * W * C * 2 + 27 * C * C * 2  # 6 input frames + 4 output + weights


def main(out):
    vals = defaultdict(dict)
    dur = defaultdict(int)
    for f in sorted(glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        span, name = {}, {}
        for r in csv.DictReader(open(f)):
            k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if k is None:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            span[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            name[d] = k
        for k in KERNELS:
            ds = [d for d in per if name[d] == k]
            if ds:
                vals[k].update(per[max(ds)])
                dur[k] = max(dur[k], span[max(ds)])
    res = {"shape": f"{C}->{C} 3x3x3, {H}x{W}, {TOUT} output frames", "flop": FLOP, "algorithmic_bytes": ALGO}
    for k, label in KERNELS.items():
        v, ns = vals.get(k, {}), dur.get(k, 0)
        if not v:
            continue
        r = {"kernel": label, "duration_ms_pmc_pass": ns / 1e6, "tflops_at_pass": FLOP / (ns / 1e9) / 1e12}
        if "FETCH_SIZE" in v:
            r["hbm_read_bytes"] = 2 * v["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in v:
            r["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in r and "hbm_write_bytes" in r:
            r["traffic_over_algorithmic"] = (r["hbm_read_bytes"] + r["hbm_write_bytes"]) / ALGO
        if "GRBM_GUI_ACTIVE" in v:
            cyc = v["GRBM_GUI_ACTIVE"] / 8
            clk = cyc / (ns / 1e9)
            r["clock_ghz"] = clk / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
                r["mfma_busy_frac"] = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
        for c in ("SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"):
            if c in v:
                r[c] = v[c]
        if "SQ_WAVE_CYCLES" in v:
            w = v["SQ_WAVE_CYCLES"]
            r["wave_split"] = {n: v[c] / w for n, c in (("active", "SQ_ACTIVE_INST_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"))
                               if c in v}
        res[k] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_conv")
