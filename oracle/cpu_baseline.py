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
The query slice is processed in chunks of 1 024 queries (the fp32 score matrix of one chunk is 7 GB at L = 109 120).
config1_end_to_end() times BASELINE config 1 whole on the CPU: the oracle's Image2World at
256 x 256 x 9 frames, 2 Karras UniPC steps (3 evaluations x CFG 2) of the 2B net, VAE encode of the conditioning
frame and decode of the 3 latent frames.
"""
from __future__ import annotations

import dataclasses
import os
import time

import torch
import torch.nn.functional as F

from .dit import apply_rope


def _rms(x, eps=1e-6):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)


def host_threads(requested: int | None = None) -> tuple[int, int]:
    """(threads to use, host cores visible to this process): the affinity mask's size, capped by OMP_NUM_THREADS (the
    GPU box's CPU share: its affinity shows the whole machine) and by an explicit request."""
    visible = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", visible) or visible)
    n = min(visible, cap)
    if requested:
        n = min(n, requested)
    return max(1, n), visible


def dit_block_sample(L: int = 109120, D: int = 2048, H: int = 16, n_q: int = 4096, ctx_len: int = 512,
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

    # ---- per-query slice (the attention in chunks of 1 024 queries)
    t0 = time.perf_counter()
    hq = h[:n_q]
    q = _rms((hq @ Wq.t()).view(n_q, H, hd))
    q = apply_rope(q[None], freqs[:n_q])[0]
    o = torch.empty(n_q, H, hd)
    for c0 in range(0, n_q, 1024):
        att = torch.softmax(torch.einsum("qhd,khd->hqk", q[c0:c0 + 1024], k) * hd ** -0.5, -1)
        o[c0:c0 + 1024] = torch.einsum("hqk,khd->qhd", att, v)
        del att
    o = o.reshape(n_q, D) @ Wo.t()
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
                   f"projections over all tokens, a {n_q}-query slice ({100.0 * n_q / L:.2f} % of the queries) of "
                   f"everything else, extrapolated x L/{n_q} x {n_blocks} blocks x {forwards} forwards; VAE excluded"),
    }


def config1_end_to_end(threads: int | None = None, seed: int = 0) -> dict:
    """BASELINE config 1 on the CPU, whole: the oracle's Image2World video at 256 x 256 x 9 frames (latent
    [16, 3, 32, 32]), 2 Karras UniPC steps with CFG (guidance 7, zeroed uncond context) of the seeded 2B net, the VAE
    encode of the conditioning frame and the decode of all 9 frames (bf16 activations as the reference runs them).
    Weight construction is not timed."""
    from cosmos_predict2.dit import init_state_dict  # seeded weights with the 2B shapes (the bench's own init)
    from cosmos_predict2.net_config import DIT_2B
    from cosmos_predict2.vae import init_vae_state_dict

    from . import sampler as osamp
    from . import vae as ovae

    if threads is not None:
        torch.set_num_threads(threads)
    sd = {"net." + k: v for k, v in init_state_dict(DIT_2B, seed=11, zero_adaln_out=False).items()}
    vsd = init_vae_state_dict(seed=0)
    g = torch.Generator().manual_seed(seed)
    img = torch.rand(1, 3, 1, 256, 256, generator=g) * 2 - 1
    ctx_c = torch.randn(1, 512, DIT_2B.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    ctx_u = torch.zeros_like(ctx_c)
    t0 = time.perf_counter()
    lat0 = ovae.encode(vsd, img)  # [1, 16, 1, 32, 32]
    gt = torch.zeros(1, 16, 3, 32, 32)
    gt[:, :, :1] = lat0.float()
    t1 = time.perf_counter()
    lat = osamp.generate(dataclasses.asdict(DIT_2B), sd, gt, ctx_c, ctx_u, num_cond=1, guidance=7.0, seed=0,
                         num_steps=2, use_karras=True, cond_frame_t=0.1)
    t2 = time.perf_counter()
    video = ovae.decode(vsd, lat)
    t3 = time.perf_counter()
    assert video.shape[2] == 9 and torch.isfinite(video.float()).all()
    return {"frames_per_s": 9 / (t3 - t0), "seconds": t3 - t0, "encode_s": t1 - t0, "sampler_s": t2 - t1,
            "decode_s": t3 - t2, "cores": torch.get_num_threads(),
            "sample": "BASELINE config 1 whole on the CPU: oracle Image2World 256x256x9f, 2B net, 2 Karras UniPC steps "
                      "(3 evals x CFG 2), VAE encode of the conditioning frame + decode of 9 frames"}
