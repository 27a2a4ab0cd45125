"""Which operand layout hipBLASLt runs fastest for the DiT projections (same FLOP, same bf16 data).

y[M, N] = x[M, K] W[N, K]^T as F.linear (weights [N, K], the checkpoint layout), as x @ Wt with the
weights stored transposed [K, N], and as (W x^T)^T (the transposed problem). Prints ms per layout.
usage: python tools/gemm_layout.py [--rows 218240]
"""
import argparse
import json

import torch
import torch.nn.functional as F

D = 2048


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=218240)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    m = a.rows
    for (n, k) in [(3 * D, D), (D, D), (4 * D, D), (D, 4 * D)]:
        x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
        wt = w.t().contiguous()
        r = {"M": m, "N": n, "K": k,
             "linear_ms": timed(lambda: F.linear(x, w)),
             "x_at_wt_ms": timed(lambda: torch.mm(x, wt)),
             "w_at_xt_ms": timed(lambda: torch.mm(w, x.t()))}
        y0 = F.linear(x, w).float()
        r["max_rel_diff_x_at_wt"] = float((torch.mm(x, wt).float() - y0).norm() / y0.norm())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
