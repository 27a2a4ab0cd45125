"""CPU baseline for bench.py — TEST INFRASTRUCTURE (see oracle/__init__.py).

The reference's own CPU path cannot run (hard-coded .cuda(), transformer-engine / flash-attn, and
the import refusal of SURVEY.md §8(c)), so the baseline is this oracle's restatement of one 2B DiT
Block.forward (minimal_v4_dit.py:1124-1247) in PyTorch-CPU fp32, timed on a bounded sample and
extrapolated (BASELINE.md "CPU-baseline plan"):
  * the parts that need every token — AdaLN-modulated LayerNorm and the K/V projections + k-norm +
    RoPE over all L tokens — run in full;
  * everything per query token — Q projection, self-attention of an `n_q`-query slice against all L
    keys, output projection, cross-attention over 512 text tokens, MLP — runs on the slice and is
    scaled by L / n_q;
  * one forward = 28 blocks; one video = 72 forwards (36 Karras evaluations x CFG 2). The VAE
    (~0.5 % of the FLOPs) is not included.
"""
from __future__ import annotations

import time

import torch
import torch.nn.functional as F

from .dit import apply_rope


def _rms(x, eps=1e-6):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)


def dit_block_sample(L: int = 109120, D: int = 2048, H: int = 16, n_q: int = 1024, ctx_len: int = 512,
                     n_blocks: int = 28, forwards: int = 72, frames: int = 121, threads: int | None = None,
                     seed: int = 0) -> dict:
    if threads is not None:
        torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(seed)
    hd = D // H
    s = D ** -0.5

    def w(o, i):
        return torch.randn(o, i, generator=g) * (i ** -0.5)

    x = torch.randn(L, D, generator=g)
    Wq, Wk, Wv, Wo = w(D, D), w(D, D), w(D, D), w(D, D)
    Wqc, Woc = w(D, D), w(D, D)
    W1, W2 = w(4 * D, D), w(D, 4 * D)
    kc = torch.randn(ctx_len, H, hd, generator=g)
    vc = torch.randn(ctx_len, H, hd, generator=g)
    shift, scale, gate = (0.1 * torch.randn(3, D, generator=g)).unbind(0)
    freqs = torch.rand(L, hd, generator=g) * 10

    # ---- full-sequence part
    t0 = time.perf_counter()
    h = F.layer_norm(x, (D,), eps=1e-6) * (1 + scale) + shift
    k = _rms((h @ Wk.t()).view(L, H, hd))
    k = apply_rope(k[None], freqs)[0]
    v = (h @ Wv.t()).view(L, H, hd)
    t_full = time.perf_counter() - t0

    # ---- per-query slice
    t0 = time.perf_counter()
    hq = h[:n_q]
    q = _rms((hq @ Wq.t()).view(n_q, H, hd))
    q = apply_rope(q[None], freqs[:n_q])[0]
    att = torch.softmax(torch.einsum("qhd,khd->hqk", q, k) * hd ** -0.5, -1)
    o = torch.einsum("hqk,khd->qhd", att, v).reshape(n_q, D) @ Wo.t()
    xs = x[:n_q] + gate * o
    h2 = F.layer_norm(xs, (D,), eps=1e-6) * (1 + scale) + shift
    qc = _rms((h2 @ Wqc.t()).view(n_q, H, hd))
    attc = torch.softmax(torch.einsum("qhd,khd->hqk", qc, kc) * hd ** -0.5, -1)
    oc = torch.einsum("hqk,khd->qhd", attc, vc).reshape(n_q, D) @ Woc.t()
    xs = xs + gate * oc
    h3 = F.layer_norm(xs, (D,), eps=1e-6) * (1 + scale) + shift
    xs = xs + gate * (F.gelu(h3 @ W1.t()) @ W2.t())
    t_slice = time.perf_counter() - t0
    del s, xs

    block_s = t_full + t_slice * (L / n_q)
    video_s = block_s * n_blocks * forwards
    return {
        "value": frames / video_s,
        "unit": "frames/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "block_seconds_extrapolated": block_s,
        "sample_seconds": t_full + t_slice,
        "sample": (f"oracle fp32 PyTorch-CPU restatement of one 2B DiT block at L={L} (720p x 121f): LN + K/V "
                   f"projections over all tokens, a {n_q}-query slice of everything else, extrapolated x L/{n_q} "
                   f"x {n_blocks} blocks x {forwards} forwards; VAE excluded"),
    }
