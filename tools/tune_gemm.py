"""Offline GEMM solution search for the DiT projections (PyTorch TunableOp over hipBLASLt/rocBLAS).

The DiT's nn.Linear calls (QKV, output projections, cross-attention q/o, MLP in/out) are plain
library GEMMs on hipBLASLt. Its default heuristic picks one kernel per shape; TunableOp times every
candidate solution on the device and records the fastest per (transposes, M, N, K). This tool runs
that search once for the token counts of CP = 1/2/4/8 (B = 2 at CP = 1, one CFG lane of B = 1
otherwise), writes the result file, and prints default-vs-tuned time per shape. The product reads
the committed file with tuning OFF (`cosmos_predict2/_native.py: enable_tuned_gemms`).

usage: python tools/tune_gemm.py --out gpurun_out/tunableop_gfx950.csv [--rows 218240,54560,...]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

D = 2048
# (N, K) of the per-block projections: QKV, self/cross output + cross q, MLP in, MLP out
NK = [(3 * D, D), (D, D), (4 * D, D), (D, 4 * D)]


def time_linear(x, w, iters=5):
    F.linear(x, w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        F.linear(x, w)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--rows", default="218240,54560,27280,13640")
    ap.add_argument("--max-ms", type=int, default=40, help="per-solution tuning budget (ms)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    rows = [int(r) for r in a.rows.split(",")]
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [(m, n, k) for m in rows for (n, k) in NK]
    base = {}
    for (m, n, k) in shapes:
        x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
        base[(m, n, k)] = time_linear(x, w)
        print(f"default M={m} N={n} K={k}: {base[(m, n, k)]:.3f} ms", flush=True)
    T = torch.cuda.tunable
    T.enable(True)
    T.tuning_enable(True)
    T.set_max_tuning_duration(a.max_ms)
    T.set_max_tuning_iterations(20)
    T.set_filename(a.out)
    for (m, n, k) in shapes:
        t0 = time.time()
        x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
        F.linear(x, w)
        torch.cuda.synchronize()
        print(f"tuned M={m} N={n} K={k} in {time.time() - t0:.1f} s", flush=True)
    T.tuning_enable(False)  # the table is written to --out when the process exits
    out = []
    for (m, n, k) in shapes:
        x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
        ms = time_linear(x, w)
        fl = 2.0 * m * n * k
        r = {"M": m, "N": n, "K": k, "default_ms": base[(m, n, k)], "tuned_ms": ms,
             "default_tflops": fl / base[(m, n, k)] / 1e9, "tuned_tflops": fl / ms / 1e9}
        out.append(r)
        print(json.dumps(r), flush=True)
    # one block: QKV, 3 x (D, D) (self output, cross q, cross output), MLP in, MLP out
    mult = {(3 * D, D): 1, (D, D): 3, (4 * D, D): 1, (D, 4 * D): 1}
    tot_d = sum(r["default_ms"] * mult[(r["N"], r["K"])] for r in out if r["M"] == rows[0])
    tot_t = sum(r["tuned_ms"] * mult[(r["N"], r["K"])] for r in out if r["M"] == rows[0])
    print(json.dumps({"rows": rows[0], "block_gemm_default_ms": tot_d, "block_gemm_tuned_ms": tot_t}), flush=True)
    print("results file:", a.out, os.path.getsize(a.out) if os.path.exists(a.out) else -1, file=sys.stderr)


if __name__ == "__main__":
    main()
