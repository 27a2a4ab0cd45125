"""Summarise tools/pmc_attn.sh / tools/pmc_passes.sh passes for one kernel (its longest, i.e. timed, dispatch).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) is doubled on gfx950 for 16-B/lane
streaming reads; WRITE_SIZE (KiB) is exact for 16-B streaming stores. Prints one JSON object.
usage: python tools/pmc_summary.py gpurun_out/pmc                      (the DiT self-attention at the bench shape)
       python tools/pmc_summary.py <dir> --kernel <substr> --flop F --algo-bytes A --name "..."   (any other kernel)
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("attn_fwd_d128<0", "attn_fwd_1w<0", "attn_fwd_m16<0")  # self-attention instantiations (d128 <0, true>: bounded shift)
FLOP = 4.0 * 2 * 16 * 109120 * 109120 * 128
ALGO_BYTES = 4 * 2 * 16 * 109120 * 128 * 2  # Q, K, V read once, O written once (bf16)


def load(out, kernels=KERNELS):
    vals, dur = {}, {}
    for f in sorted(glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        span = {}
        for r in csv.DictReader(open(f)):
            if not any(k in r["Kernel_Name"] for k in kernels):
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            span[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if per:
            # the longest dispatch: the timed launch (tail-split segments and small correctness launches share names)
            last = max(per, key=lambda d: span[d])
            vals.update(per[last])
            dur[os.path.basename(f)] = span[last]
    return vals, dur


def main(out, kernels=KERNELS, name="cp25_attn_fwd self-attention B=2 H=16 L=109120", flop=FLOP, algo=ALGO_BYTES):
    v, dur = load(out, kernels)
    ns = max(dur.values())
    res = {"kernel": name, "duration_ms_pmc_pass": ns / 1e6}
    if "FETCH_SIZE" in v:
        res["hbm_read_bytes"] = 2 * v["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in v:
        res["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
    if "hbm_read_bytes" in res and "hbm_write_bytes" in res:
        res["traffic_bytes_per_launch"] = res["hbm_read_bytes"] + res["hbm_write_bytes"]
        res["algorithmic_bytes_per_launch"] = algo
    if "GRBM_GUI_ACTIVE" in v:
        clk = v["GRBM_GUI_ACTIVE"] / 8 / (ns / 1e9)
        res["clock_ghz"] = clk / 1e9
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
            res["mfma_busy_frac"] = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
        res["tflops_at_pass"] = flop / (ns / 1e9) / 1e12
        res["peak_at_clock_tflops"] = 1024 * 1024 * clk / 1e12
    if "SQ_WAVE_CYCLES" in v:
        w = v["SQ_WAVE_CYCLES"]
        res["wave_split"] = {k: v[c] / w for k, c in (("active", "SQ_ACTIVE_INST_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"),
                                                   ("wait", "SQ_WAIT_ANY")) if c in v}
    for c in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT"):
        if c in v:
            res[c] = v[c]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--name", default="")
    ap.add_argument("--flop", type=float, default=FLOP)
    ap.add_argument("--algo-bytes", type=float, default=ALGO_BYTES)
    a = ap.parse_args()
    if a.kernel:
        main(a.out, (a.kernel,), a.name or a.kernel, a.flop, a.algo_bytes)
    else:
        main(a.out)
