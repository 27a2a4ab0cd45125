"""A/B of the text cross-attention's two kernel forms at the DiT's launch (interleaved, HIP events on the launch stream).

usage: python tools/bench_xattn.py [--L 109120] [--B 2] [--H 16] [--Lk 512] [--rounds 3] [--iters 20]
Form 1 = persistent (attn_fwd_m16<cross, .., persistent>), 0 = one workgroup per query block. q is token-major
([L, B, H*128] as the DiT's cross-attention q buffer), RMS-normed rows with the DiT's unit-weight bounds (zero shift)
and, with --online, without bounds (online max). Prints one JSON line per (form, round): ms per launch, TFLOP/s
(4 B H L Lk 128 algorithmic FLOP) and the fraction of the 2.5 PF bf16 dense peak.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

LOG2E = 1.4426950408889634


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=109120)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--Lk", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--online", action="store_true", help="no norm bounds: the online-max mode")
    ap.add_argument("--lib", default="", help="lab build of libcp25.so (tools/lab/attn_variant.py)")
    ap.add_argument("--forms", default="1,0", help="forms to time, in order")
    args = ap.parse_args()
    if args.lib:
        N._LIB_PATH = args.lib
    dev = torch.device("cuda:0")
    B, H, L, Lk = args.B, args.H, args.L, args.Lk
    g = torch.Generator(device="cpu").manual_seed(0)
    nb = 128 ** 0.5  # unit RMSNorm weights: |row| = sqrt(128)
    q = torch.nn.functional.normalize(torch.randn(L, B, H, 128, generator=g), dim=-1) * nb * (128 ** -0.5 * LOG2E)
    q = q.to(dev, torch.bfloat16).transpose(0, 1)
    k = (torch.nn.functional.normalize(torch.randn(B, Lk, H, 128, generator=g), dim=-1) * nb).to(dev, torch.bfloat16)
    v = torch.randn(B, Lk, H, 128, generator=g).to(dev, torch.bfloat16)
    o = torch.empty(L, B, H, 128, dtype=torch.bfloat16, device=dev).transpose(0, 1)
    bounds = None if args.online else (nb * 1.02 * 128 ** -0.5 * LOG2E, nb * 1.02)
    flop = 4.0 * B * H * L * Lk * 128
    stream = torch.cuda.current_stream(dev)
    forms = [int(f) for f in args.forms.split(",")]
    for form in forms:
        N.attn_cross_select(form)
        N.attn_fwd(q, k, v, out=o, prescaled=True, norm_bounds=bounds, n_split=1)
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for form in forms:
            N.attn_cross_select(form)
            name = N.attn_kernel_name(Lk, norm_bounds=bounds, prescaled=True)
            for _ in range(3):
                N.attn_fwd(q, k, v, out=o, prescaled=True, norm_bounds=bounds, n_split=1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.iters):
                N.attn_fwd(q, k, v, out=o, prescaled=True, norm_bounds=bounds, n_split=1)
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            print(json.dumps({"lib": os.path.basename(args.lib) or "product", "round": r, "form": form, "kernel": name, "B": B, "H": H, "L": L, "Lk": Lk,
                              "ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1),
                              "frac_of_2500": round(flop / ms / 1e9 / 2500, 3)}), flush=True)
    N.attn_cross_select(1)


if __name__ == "__main__":
    main()
