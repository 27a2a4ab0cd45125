"""The projections whose head norm moved into the GEMM epilogue, at the metric shape (M = 218 240): the cross-attention
q (2048 x 2048; cp25_gemm_epi + cp25_head_rmsnorm_rope_scaled vs cp25_gemm_hnorm) and the fused QKV (6144 x 2048;
cp25_gemm_epi + the k RMSNorm + RoPE pass vs cp25_gemm_qkv), HIP events, interleaved rounds in one process. One JSON
line per projection.
usage: python tools/bench_hnorm.py [--rounds 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402


def timed(fn, iters=5):
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
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M, D = 218240, 2048
    x = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(D, D, device=dev, generator=g) * D ** -0.5).to(torch.bfloat16)
    nw = (0.5 + torch.rand(128, device=dev, generator=g)).to(torch.bfloat16)
    out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    c = 128 ** -0.5 * 1.4426950408889634

    def two_pass():
        N.gemm_epi(x, w, out=out)
        N.head_rmsnorm_rope(out, n_rows=M, B=1, H=D // 128, head_off=0, weight=nw, out_scale=c)

    def fused():
        N.gemm_hnorm(x, w, nw, out_scale=c, out=out)

    res = {"two_pass_ms": [], "fused_ms": [], "gemm_only_ms": []}
    for _ in range(a.rounds):
        res["two_pass_ms"].append(timed(two_pass))
        res["fused_ms"].append(timed(fused))
        res["gemm_only_ms"].append(timed(lambda: N.gemm_epi(x, w, out=out)))
    print(json.dumps({"proj": "cross-q", "shape": f"M={M} N={D} K={D}", **res, "min_two_pass": min(res["two_pass_ms"]),
                      "min_fused": min(res["fused_ms"]), "min_gemm_only": min(res["gemm_only_ms"])}), flush=True)
    # the QKV projection: k columns normed + RoPE (B = 2 token-major rows)
    w3 = (torch.randn(3 * D, D, device=dev, generator=g) * D ** -0.5).to(torch.bfloat16)
    out3 = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    ang = torch.rand(M // 2, 64, device=dev, generator=g) * 50.0
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()

    def two_pass3():
        N.gemm_epi(x, w3, out=out3)
        N.head_rmsnorm_rope(out3, n_rows=M, B=2, H=D // 128, head_off=D, weight=nw, cos=cos, sin=sin)

    def fused3():
        N.gemm_qkv(x, w3, nw, k_col0=D, k_cols=D, B=2, cos=cos, sin=sin, out=out3)

    res = {"two_pass_ms": [], "fused_ms": [], "gemm_only_ms": []}
    for _ in range(a.rounds):
        res["two_pass_ms"].append(timed(two_pass3))
        res["fused_ms"].append(timed(fused3))
        res["gemm_only_ms"].append(timed(lambda: N.gemm_epi(x, w3, out=out3)))
    print(json.dumps({"proj": "qkv", "shape": f"M={M} N={3 * D} K={D}", **res, "min_two_pass": min(res["two_pass_ms"]),
                      "min_fused": min(res["fused_ms"]), "min_gemm_only": min(res["gemm_only_ms"])}), flush=True)


if __name__ == "__main__":
    main()
