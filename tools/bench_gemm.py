"""The DiT block projections on the hand-written GEMM vs hipBLASLt at the metric shape (M = 218 240 = 109 120 tokens x
CFG 2), HIP events, interleaved rounds in one process. One JSON line per shape:
  bf16: cp25_gemm_epi vs torch.matmul; MLP1 + GELU fused vs matmul + cp25_gelu; the gated residual fused
        (cp25_gemm_res, then the LN-mod reads x' only) vs matmul + cp25_ln_mod(x, y, gate);
  fp8 : cp25_gemm_fp8 vs torch._scaled_mm on the same row-scaled e4m3 operands (config 5's option).
usage: python tools/bench_gemm.py [--rounds 2] [--fp8] [--shapes qkv,mlp1] [--plain] [--lib tools/lab/libcp25_<x>.so]
(--plain: own vs library only, no fused comparisons; --lib: a lab build, tools/lab/gemm_variant.py)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

dev = torch.device("cuda:0")


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
    ap.add_argument("--M", type=int, default=218240)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--shapes", default="qkv,proj,mlp1,mlp2")
    ap.add_argument("--plain", action="store_true")
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    if a.lib:
        N._LIB_PATH = a.lib
    M, B, hw, T = a.M, 2, 3520, 31
    for name, Nn, K in (("qkv", 6144, 2048), ("proj", 2048, 2048), ("mlp1", 8192, 2048), ("mlp2", 2048, 8192)):
        if name not in a.shapes.split(","):
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(Nn, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * M * Nn * K
        rec = {"gemm": name, "M": M, "N": Nn, "K": K, "lib": os.path.basename(a.lib) or "libcp25.so"}
        res = {"lib": [], "own": []}
        if a.fp8:
            q, s = N.quant_fp8_rows(x)
            fmax = torch.finfo(torch.float8_e4m3fn).max
            ws = (w.float().abs().amax(1, keepdim=True) / fmax).clamp_min(1e-30)
            w8 = (w.float() / ws).clamp(-fmax, fmax).to(torch.float8_e4m3fn)
            wsr = ws.t().contiguous()
            for _ in range(a.rounds):
                res["lib"].append(timed(lambda: torch._scaled_mm(q, w8.t(), scale_a=s, scale_b=wsr,
                                                                  out_dtype=torch.bfloat16)))
                res["own"].append(timed(lambda: N.gemm_fp8(q, s, w8, wsr, out=out)))
            rec.update(kind="fp8", scaled_mm_ms=res["lib"], own_ms=res["own"],
                       scaled_mm_tflops=flop / min(res["lib"]) / 1e9, own_tflops=flop / min(res["own"]) / 1e9)
            print(json.dumps(rec), flush=True)
            continue
        for _ in range(a.rounds):
            res["lib"].append(timed(lambda: torch.matmul(x, w.t(), out=out)))
            res["own"].append(timed(lambda: N.gemm_epi(x, w, out=out)))
        rec.update(kind="bf16", hipblaslt_ms=res["lib"], own_ms=res["own"],
                   hipblaslt_tflops=flop / min(res["lib"]) / 1e9, own_tflops=flop / min(res["own"]) / 1e9)
        if a.plain:
            print(json.dumps(rec), flush=True)
            continue
        if name == "mlp1":
            def unfused():
                torch.matmul(x, w.t(), out=out)
                N.gelu_(out)
            rec["lib_plus_gelu_ms"] = min(timed(unfused) for _ in range(a.rounds))
            rec["own_gelu_fused_ms"] = min(timed(lambda: N.gemm_epi(x, w, epilogue=N.EPI_GELU, out=out))
                                           for _ in range(a.rounds))
        if Nn == 2048:
            # the sub-layer's output projection + gated residual + the next LN-mod, both ways
            n = M // B
            xr = torch.randn(n, B, Nn, device=dev, generator=g).to(torch.bfloat16)
            mods = torch.randn(B, T, 3 * Nn, device=dev, generator=g).to(torch.bfloat16)
            sh, sc, gate = mods[..., :Nn], mods[..., Nn:2 * Nn], mods[..., 2 * Nn:]
            xo = torch.empty_like(xr)
            kw = dict(n_tok=n, B=B, tok0=0, hw=hw)

            def lib_res():
                torch.matmul(x, w.t(), out=out)
                N.ln_mod(xr, sh, sc, x_st=B * Nn, x_sb=Nn, y=out, gate=gate, x_out=xo, **kw)

            def own_res():
                N.gemm_res(x, w, xr, B * Nn, Nn, gate, B=B, tok0=0, hw=hw, out=xo.view(M, Nn))
                N.ln_mod(xo, sh, sc, x_st=B * Nn, x_sb=Nn, **kw)

            rec["lib_plus_ln_mod_residual_ms"] = min(timed(lib_res) for _ in range(a.rounds))
            rec["own_residual_fused_plus_ln_mod_ms"] = min(timed(own_res) for _ in range(a.rounds))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
