"""Default vs committed-table GEMM time for the DiT block projections (same process, same inputs).

usage: python tools/gemm_check.py --table gpurun_out/tunableop_gfx950.csv [--rows 218240,13640]
Prints one JSON line per (M, N, K) with both times and the rel-L2 between the two results.
"""
import argparse
import json
import os
import sys


import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


D = 2048


def timed(x, w, iters=10):
    y = F.linear(x, w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        F.linear(x, w)
    e1.record()
    torch.cuda.synchronize()
    return y, e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="218240,13640")
    ap.add_argument("--table", required=True, help="TunableOp results file from tools/tune_gemm.py")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    mult = {(3 * D, D): 1, (D, D): 3, (4 * D, D): 1, (D, 4 * D): 1}
    cases = []
    for m in [int(r) for r in a.rows.split(",")]:
        for (n, k) in mult:
            x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
            cases.append((m, n, k, x, w))
    base = [timed(x, w) for (_, _, _, x, w) in cases]
    T = torch.cuda.tunable
    T.enable(True)
    T.tuning_enable(False)
    on = bool(T.read_file(a.table))
    tot = {}
    for (m, n, k, x, w), (y0, t0) in zip(cases, base):
        y1, t1 = timed(x, w)
        rel = float((y1.float() - y0.float()).norm() / y0.float().norm())
        fl = 2.0 * m * n * k
        print(json.dumps({"M": m, "N": n, "K": k, "default_ms": t0, "tuned_ms": t1, "default_tflops": fl / t0 / 1e9,
                          "tuned_tflops": fl / t1 / 1e9, "rel_l2": rel}), flush=True)
        d = tot.setdefault(m, [0.0, 0.0])
        d[0] += t0 * mult[(n, k)]
        d[1] += t1 * mult[(n, k)]
        assert rel < 1e-2, rel
    print(json.dumps({"table_active": on, "block_gemm_ms_default_vs_tuned": tot}), flush=True)
    if not on:
        sys.exit(1)


if __name__ == "__main__":
    main()
