"""Lab A/B: every bf16 GEMM epilogue (plain, GELU, head-norm, q|k|v with k norm + RoPE, gated residual) of the
current libcp25.so against tools/lab/gemm_tail/libcp25_base.so (gemm.hip before the tail row slices) at the metric
shape (M = 218 240) and a CP = 8 lane's (13 640), alternating in one process by swapping _native's library handle.
One JSON line per (M, epilogue): min ms of 4 alternating rounds, bit-identity of the two outputs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

dev = torch.device("cuda:0")
new = N.load_library()
N._lib, N._LIB_PATH = None, os.path.join(ROOT, "tools/lab/gemm_tail/libcp25_base.so")
base = N.load_library()
libs = {"new": new, "base": base}


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


g = torch.Generator(device=dev).manual_seed(0)
for M in (218240, 13640):
    B = 2 if M == 218240 else 1
    n_tok, hw = M // B, 3520
    D = 2048
    x = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    x4 = torch.randn(M, 4 * D, device=dev, generator=g).to(torch.bfloat16)
    nw = (0.5 + torch.rand(128, device=dev, generator=g)).to(torch.bfloat16)
    wq = (torch.randn(D, D, device=dev, generator=g) * D ** -0.5).to(torch.bfloat16)
    wqkv = (torch.randn(3 * D, D, device=dev, generator=g) * D ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(D, 4 * D, device=dev, generator=g) * (4 * D) ** -0.5).to(torch.bfloat16)
    xr = torch.randn(n_tok, B, D, device=dev, generator=g).to(torch.bfloat16)
    T = -(-n_tok // hw)
    gate = torch.randn(B, T, 3 * D, device=dev, generator=g).to(torch.bfloat16)[..., 2 * D:]
    ang = torch.rand(n_tok, 64, device=dev, generator=g) * 30
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    cases = {
        "hnorm": lambda: N.gemm_hnorm(x, wq, nw, out_scale=0.127),
        "qkv": lambda: N.gemm_qkv(x, wqkv, nw, k_col0=D, k_cols=D, B=B, cos=cos, sin=sin),
        "res_mlp2": lambda: N.gemm_res(x4, w2, xr, B * D, D, gate, B=B, tok0=0, hw=hw),
        "res_proj": lambda: N.gemm_res(x, wq, xr, B * D, D, gate, B=B, tok0=0, hw=hw),
    }
    for name, fn in cases.items():
        outs, t = {}, {"new": [], "base": []}
        for r in range(4):
            for which in (("new", "base") if r % 2 == 0 else ("base", "new")):
                N._lib = libs[which]
                outs[which] = fn()
                t[which].append(round(timed(fn), 4))
        print(json.dumps({"M": M, "gemm": name, "bit_identical": bool(torch.equal(outs["new"], outs["base"])),
                          "new_ms": t["new"], "base_ms": t["base"], "new_min": min(t["new"]), "base_min": min(t["base"]),
                          "base_over_new": min(t["base"]) / min(t["new"])}), flush=True)
N._lib = new
