"""DiT denoiser forward restatement (CPU) — TEST INFRASTRUCTURE (see oracle/__init__.py).

Restates MinimalV1LVGDiT.forward -> MiniTrainDIT.forward as the reference runs it at inference:
net weights and float buffers in bf16 (utils/model_loader.py:88-90 + on_train_start), bf16 torch ops
for the block body, fp32 autocast for the t-embedding, AdaLN modulation and final layer
(use_wan_fp32_strategy, minimal_v4_dit.py:974-995, 1136-1154, 1615-1619), q/k upcast to fp32 for
RoPE (:415-419) and recast to bf16 by attention() (networks/attention.py:107-109).
Nets with use_wan_fp32_strategy=False (the multi-view nets, predict2_multiview/configs/vid2vid/defaults/net.py:52,
105) run those layers without the autocast, in the net's bf16 (multiview_dit.py:544-548, multiview_cross_dit.py:334,
823-835), with the timesteps in the net dtype (the cast video2world_model.py:231-236 applies when the flag is off;
the rectified-flow denoise passes fp32 timesteps, which the bf16 TimestepEmbedding.linear_1 cannot take without the
autocast, minimal_v4_dit.py:776). Their RoPE skips the fp32 upcast (:415-419), but TE's fused RoPE computes in fp32
and rounds once to the input dtype, which is where attention() rounds the upcast q / k: the same values either way.

Paths relative to cosmos_predict2/_src/predict2/networks/ unless stated:
  minimal_v1_lvg_dit.py:31-62      condition-mask channel, timestep scale
  minimal_v4_dit.py:1517-1565      padding mask + PatchEmbed (:846-913)
  minimal_v4_dit.py:539-667        3D RoPE (bf16 range buffers, F8)
  minimal_v4_dit.py:727-788        Timesteps / TimestepEmbedding (adaln-lora)
  minimal_v4_dit.py:1124-1247      Block.forward
  minimal_v4_dit.py:916-995        FinalLayer
  minimal_v4_dit.py:1567-1575      unpatchify
Third-party numerics restated by their standard formulas (parity unpinned):
TE RMSNorm (fp32 math, one rounding of (x*rstd)*w), TE fused RoPE (rotate-half, fp32), SDPA
(fp32 softmax, bf16 output; or, inside `flash_sdpa()`, the flash-attention forward's bf16-P numerics).

Config: a dict with the DiTConfig field names (cosmos_predict2/net_config.py).
Device-agnostic torch code: the tests run it on the CPU, and at full-geometry sizes that would take hours on host
cores (a 136 080-token multi-view block) on the GPU's own torch ops (fp32 matmuls), never on this repository's
kernels.
Weights: a state dict with the reference's `net.` key layout, bf16 tensors.
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16
F32 = torch.float32

# activation dtype of the restatement: bf16 = the reference's inference arithmetic; fp32 (inside
# `fp32_truth()`) = the same bf16-valued weights with every activation kept in fp32 (no intermediate
# bf16 rounding), the "truth" both the bf16 reference and the HIP path are measured against
_ACT = [BF16]


def act_dtype() -> torch.dtype:
    return _ACT[-1]


@contextlib.contextmanager
def fp32_truth():
    _ACT.append(F32)
    try:
        yield
    finally:
        _ACT.pop()


def _w(sd, name):
    w = sd["net." + name]
    return w.float() if _ACT[-1] == F32 else w


def te_rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return ((xf * rstd) * w.float()).to(x.dtype)


def rope_freqs(cfg: dict, T: int, H: int, W: int, device="cpu") -> torch.Tensor:
    """VideoRopePosition3DEmb.generate_embeddings with bf16 buffers -> [T*H*W, 128] fp32."""
    dim = cfg["model_channels"] // cfg["num_heads"]
    dim_h = dim // 6 * 2
    dim_t = dim - 2 * dim_h
    # buffers (registered fp32, cast to bf16 with the net)
    spatial_range = (torch.arange(0, dim_h, 2)[: dim_h // 2].float() / dim_h).to(BF16)
    temporal_range = (torch.arange(0, dim_t, 2)[: dim_t // 2].float() / dim_t).to(BF16)
    len_h = cfg["max_img_h"] // cfg["patch_spatial"]
    len_w = cfg["max_img_w"] // cfg["patch_spatial"]
    len_t = cfg["max_frames"] // cfg["patch_temporal"]
    seq = torch.arange(max(len_h, len_w, len_t)).float().to(BF16)
    h_theta = 10000.0 * cfg["rope_h_extrapolation_ratio"] ** (dim_h / (dim_h - 2))
    w_theta = 10000.0 * cfg["rope_w_extrapolation_ratio"] ** (dim_h / (dim_h - 2))
    t_theta = 10000.0 * cfg["rope_t_extrapolation_ratio"] ** (dim_t / (dim_t - 2))
    fh = 1.0 / (h_theta ** spatial_range.float())
    fw = 1.0 / (w_theta ** spatial_range.float())
    ft = 1.0 / (t_theta ** temporal_range.float())
    eh = torch.outer(seq[:H], fh)
    ew = torch.outer(seq[:W], fw)
    et = torch.outer(seq[:T], ft)
    grid = torch.cat(
        [
            et[:, None, None, :].expand(T, H, W, -1),
            eh[None, :, None, :].expand(T, H, W, -1),
            ew[None, None, :, :].expand(T, H, W, -1),
        ]
        * 2,
        dim=-1,
    )
    return grid.reshape(T * H * W, dim).float().to(device)


def apply_rope(x: torch.Tensor, freqs: torch.Tensor) -> torch.Tensor:
    """rotate-half RoPE in fp32: x [B, L, H, D] fp32, freqs [L, D]."""
    d2 = x.shape[-1] // 2
    rot = torch.cat([-x[..., d2:], x[..., :d2]], dim=-1)
    c = torch.cos(freqs)[None, :, None, :]
    s = torch.sin(freqs)[None, :, None, :]
    return x * c + rot * s


# SDPA form of the bf16 restatement: "fp32p" (default) keeps the softmax weights P in fp32 through P.V (more exact
# than any kernel the reference dispatches to); "flash" (inside `flash_sdpa()`) restates the flash-attention forward
# those kernels run (networks/attention.py:119-178 dispatches to FlashAttention-3 / cuDNN SDPA / FlashAttention-2;
# third-party, not vendored in the reference: FlashAttention-2, Dao 2023, Algorithm 1, as in its csrc
# flash_fwd_kernel.h / softmax.h): key blocks of 128, a running row max m_j over the blocks seen so far, P_j =
# exp2(S_j * scale * log2 e - m_j * scale * log2 e) in fp32, the row sum l over the UNROUNDED fp32 P, P_j rounded to
# bf16 for the P.V product (fp32 accumulation), O rescaled by exp2 of the max change, O / l rounded once to bf16.
# Parity unpinned (no fixture of those kernels exists here); it measures the bf16-P floor between two flash-class
# implementations.
_SDPA = ["fp32p"]


@contextlib.contextmanager
def flash_sdpa():
    _SDPA.append("flash")
    try:
        yield
    finally:
        _SDPA.pop()


def _flash_rows(qf: torch.Tensor, kf: torch.Tensor, vf: torch.Tensor, scale: float, blk: int = 128) -> torch.Tensor:
    """FlashAttention-2 forward numerics on [B, H, q, D] fp32 q (bf16-valued) against [B, H, Lk, D] k / v: the key
    blocks are processed in order with the running max (vectorised: the max seen through block j is the cumulative
    max of the block maxima; the sequential rescales of O and l multiply to exp2(m_j - m_final) per block)."""
    s = torch.matmul(qf, kf.transpose(-1, -2))  # raw scores, fp32
    Lk = s.shape[-1]
    nb = (Lk + blk - 1) // blk
    pad = nb * blk - Lk
    if pad:
        s = F.pad(s, (0, pad), value=float("-inf"))
    sb = s.view(*s.shape[:-1], nb, blk)
    c = scale * math.log2(math.e)
    m = torch.cummax(sb.amax(-1), dim=-1).values * c  # [.., q, nb] running max, log2 units
    p = torch.exp2(sb * c - m[..., None])              # fp32 P of each block at its running max
    w = torch.exp2(m - m[..., -1:])                    # rescale of block j to the final max
    l = (p.sum(-1) * w).sum(-1, keepdim=True)          # row sum of the unrounded P
    pw = (p.to(BF16).float() * w[..., None]).view(*s.shape[:-1], nb * blk)[..., :Lk]
    return torch.matmul(pw, vf) / l


def sdpa(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, chunk: int = 4096) -> torch.Tensor:
    """[B, S, H, D] bf16 -> [B, S, H*D] bf16 with fp32 softmax (query-chunked for memory: a chunk's fp32 scores stay
    under ~16 GB, e.g. 384 queries at config 4's 163 800 keys). Inside `flash_sdpa()`: the flash-attention numerics
    (bf16 P for P.V, _flash_rows)."""
    B, Lq, H, D = q.shape
    chunk = max(128, min(chunk, (16 << 30) // (B * H * k.shape[1] * 4) // 128 * 128))
    kf = k.float().transpose(1, 2)
    vf = v.float().transpose(1, 2)
    outs = []
    for s0 in range(0, Lq, chunk):
        qf = q[:, s0 : s0 + chunk].float().transpose(1, 2)
        if _SDPA[-1] == "flash" and act_dtype() == BF16:
            outs.append(_flash_rows(qf, kf, vf, D ** -0.5).transpose(1, 2))
            continue
        p = torch.softmax(torch.matmul(qf, kf.transpose(-1, -2)) * (D ** -0.5), dim=-1)
        outs.append(torch.matmul(p, vf).transpose(1, 2))
    o = torch.cat(outs, dim=1)
    return o.reshape(B, Lq, H * D).to(act_dtype())


def _lin(x, w, b=None):
    return F.linear(x, w, b)


def action_embedding(cfg, sd, action: torch.Tensor):
    """action_conditioned_minimal_v1_lvg_dit.py: Mlp (:28-45: fc1 + bias, GELU(tanh), fc2 + bias) in
    the model dtype (bf16) on the action [B, A, d]; per chunk (:104-107) -> [B, 1, *], per latent
    frame (:257-270) -> [B, A/r, *] with a zero row prepended for latent frame 0."""
    a = action.to(act_dtype())
    B, A, d = a.shape
    r = cfg.get("action_per_latent_frame", 0)
    a = a.reshape(B, A // r, r * d) if r else a.reshape(B, 1, A * d)

    def mlp(name):
        h = F.gelu(_lin(a, _w(sd, name + ".fc1.weight"), _w(sd, name + ".fc1.bias")), approximate="tanh")
        return _lin(h, _w(sd, name + ".fc2.weight"), _w(sd, name + ".fc2.bias"))

    e_d, e_3d = mlp("action_embedder_B_D"), mlp("action_embedder_B_3D")
    if r:
        e_d = torch.cat([torch.zeros_like(e_d[:, :1]), e_d], 1)
        e_3d = torch.cat([torch.zeros_like(e_3d[:, :1]), e_3d], 1)
    return e_d, e_3d


def cond_dtype(cfg) -> torch.dtype:
    """dtype of the t-embedding, AdaLN, view projection and final layer: fp32 (the autocast of
    use_wan_fp32_strategy, and the fp32 truth), else the net's bf16."""
    return F32 if cfg.get("use_wan_fp32_strategy", True) or act_dtype() == F32 else BF16


def timestep_embedding(cfg, sd, t_B_T: torch.Tensor, action: torch.Tensor | None = None):
    """Timesteps (fp32 sinusoid, returned in t's dtype) + TimestepEmbedding(adaln-lora) + t_embedding_norm in the
    conditioning dtype (cond_dtype); action nets add the action embeddings before the norm
    (action_conditioned_minimal_v1_lvg_dit.py:298-305)."""
    D = cfg["model_channels"]
    cd = cond_dtype(cfg)
    half = D // 2
    expo = -math.log(10000) * torch.arange(half, dtype=F32, device=t_B_T.device) / (half - 0.0)
    emb = t_B_T.flatten().float()[:, None] * torch.exp(expo)[None, :]
    sincos = torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1).reshape(t_B_T.shape[0], t_B_T.shape[1], D).to(cd)
    h = F.silu(_lin(sincos, _w(sd, "t_embedder.1.linear_1.weight").to(cd)))
    lora = _lin(h, _w(sd, "t_embedder.1.linear_2.weight").to(cd))
    if action is not None:
        e_d, e_3d = action_embedding(cfg, sd, action)
        sincos = sincos + e_d.to(cd)
        lora = lora + e_3d.to(cd)
    emb_norm = te_rmsnorm(sincos, _w(sd, "t_embedding_norm.weight"))
    return emb_norm, lora


def adaln(sd, prefix, emb, lora, n_chunks=3):
    """SiLU -> Linear(D, A) -> Linear(A, n D), + the AdaLN-LoRA term, in emb's dtype (cond_dtype)."""
    h = F.silu(emb)
    h = _lin(h, _w(sd, prefix + ".1.weight").to(emb.dtype))
    h = _lin(h, _w(sd, prefix + ".2.weight").to(emb.dtype))
    return (h + lora[..., : h.shape[-1]]).chunk(n_chunks, dim=-1)


def ln_mod(x, shift, scale):
    # nn.LayerNorm(no affine, eps 1e-6) on bf16 -> bf16, then bf16 ops (minimal_v4_dit.py:1171-1172)
    return F.layer_norm(x, (x.shape[-1],), eps=1e-6) * (1 + scale) + shift


def cross_view_attention(cfg, sd, p, x, n_views: int, view_ids) -> torch.Tensor:
    """MultiViewCrossBlock's cross-view sub-layer (predict2_multiview/networks/multiview_cross_dit.py:436-450) over
    CrossViewAttention.forward (:138-228), x [B, T, H, W, D] with the views stacked along T: the affine LayerNorm, then
    per (batch entry, latent frame, view) the view's H*W tokens attend to its neighbours' tokens of the same frame
    (neighbour ids of the view's id from the map, looked up among the input's view ids; absent ones masked, i.e.
    left out; key order: neighbour positions sorted descending, :177-186), q / k RMS-normed, no RoPE; output_proj;
    the un-gated residual. A view with no neighbour present contributes nothing (the reference's all-masked row)."""
    nh, hd = cfg["num_heads"], cfg["model_channels"] // cfg["num_heads"]
    B, T, H, W, D = x.shape
    Tv, hw = T // n_views, H * W
    xn = F.layer_norm(x, (D,), _w(sd, p + "layer_norm_cross_view_attn.weight"),
                      _w(sd, p + "layer_norm_cross_view_attn.bias"), eps=1e-6)
    xv = xn.reshape(B, n_views, Tv, hw, D)
    q = te_rmsnorm(_lin(xv, _w(sd, p + "cross_view_attn.q_proj.weight")).reshape(B, n_views, Tv, hw, nh, hd),
                   _w(sd, p + "cross_view_attn.q_norm.weight"))
    k = te_rmsnorm(_lin(xv, _w(sd, p + "cross_view_attn.k_proj.weight")).reshape(B, n_views, Tv, hw, nh, hd),
                   _w(sd, p + "cross_view_attn.k_norm.weight"))
    v = _lin(xv, _w(sd, p + "cross_view_attn.v_proj.weight")).reshape(B, n_views, Tv, hw, nh, hd)
    amap = cfg["cross_view_attn_map"]
    pos = {int(vid): j for j, vid in enumerate(view_ids)}
    o = torch.zeros(B, n_views, Tv, hw, nh * hd, dtype=act_dtype(), device=x.device)
    for j, vid in enumerate(view_ids):
        nb = sorted((pos[u] for u in amap[int(vid)] if u in pos), reverse=True) if int(vid) < len(amap) else []
        if not nb:
            continue
        kk = torch.cat([k[:, u] for u in nb], dim=2)  # [B, Tv, n_nb * hw, nh, hd]
        vv = torch.cat([v[:, u] for u in nb], dim=2)
        oj = sdpa(q[:, j].reshape(B * Tv, hw, nh, hd), kk.reshape(B * Tv, -1, nh, hd), vv.reshape(B * Tv, -1, nh, hd))
        o[:, j] = oj.reshape(B, Tv, hw, nh * hd)
    out = _lin(o, _w(sd, p + "cross_view_attn.output_proj.weight")).reshape(B, T, H, W, D)
    return x + out


def block_forward(cfg, sd, i, x, emb, lora, ctx, freqs, n_views: int = 1, view_mod=None, view_ids=None):
    """Block.forward, x [B, T, H, W, D] bf16 (multi-view: MultiViewBlock, per-view cross-attention; cross-view nets:
    MultiViewCrossBlock, multiview_cross_dit.py:313-500 -- per-view self-attention, the cross-view sub-layer, and the
    view modulation view_mod [9, T, D] bf16 added to the bf16 shift / scale / gate, :355-404)."""
    p = f"blocks.{i}."
    nh, hd = cfg["num_heads"], cfg["model_channels"] // cfg["num_heads"]
    sh_sa, sc_sa, g_sa = adaln(sd, p + "adaln_modulation_self_attn", emb, lora)
    sh_ca, sc_ca, g_ca = adaln(sd, p + "adaln_modulation_cross_attn", emb, lora)
    sh_ml, sc_ml, g_ml = adaln(sd, p + "adaln_modulation_mlp", emb, lora)
    cvt = lambda t: t[:, :, None, None, :].to(act_dtype())  # noqa: E731
    mods = [cvt(t) for t in (sh_sa, sc_sa, g_sa, sh_ca, sc_ca, g_ca, sh_ml, sc_ml, g_ml)]
    if view_mod is not None:
        mods = [m + view_mod[j][None, :, None, None, :].to(act_dtype()) for j, m in enumerate(mods)]
    sh_sa, sc_sa, g_sa, sh_ca, sc_ca, g_ca, sh_ml, sc_ml, g_ml = mods
    B, T, H, W, D = x.shape
    cross_view = bool(cfg.get("cross_view_attn_map"))

    # self attention (cross-view nets: per view, "(b v) (t h w)")
    h = ln_mod(x, sh_sa, sc_sa).reshape(B, T * H * W, D)
    q = _lin(h, _w(sd, p + "self_attn.q_proj.weight")).reshape(B, -1, nh, hd)
    k = _lin(h, _w(sd, p + "self_attn.k_proj.weight")).reshape(B, -1, nh, hd)
    v = _lin(h, _w(sd, p + "self_attn.v_proj.weight")).reshape(B, -1, nh, hd)
    q = te_rmsnorm(q, _w(sd, p + "self_attn.q_norm.weight")).float()
    k = te_rmsnorm(k, _w(sd, p + "self_attn.k_norm.weight")).float()
    q = apply_rope(q, freqs)
    k = apply_rope(k, freqs)
    if cross_view:
        sv = lambda t: t.to(act_dtype()).reshape(B * n_views, -1, nh, hd)  # noqa: E731
        o = sdpa(sv(q), sv(k), sv(v)).reshape(B, T * H * W, nh * hd)
    else:
        o = sdpa(q.to(act_dtype()), k.to(act_dtype()), v.to(act_dtype()))
    o = _lin(o, _w(sd, p + "self_attn.output_proj.weight")).reshape(B, T, H, W, D)
    x = x + g_sa * o
    if cross_view:
        x = cross_view_attention(cfg, sd, p, x, n_views, view_ids)

    # cross attention (no RoPE)
    h = ln_mod(x, sh_ca, sc_ca).reshape(B, T * H * W, D)
    q = _lin(h, _w(sd, p + "cross_attn.q_proj.weight")).reshape(B, -1, nh, hd)
    k = _lin(ctx, _w(sd, p + "cross_attn.k_proj.weight")).reshape(B, -1, nh, hd)
    v = _lin(ctx, _w(sd, p + "cross_attn.v_proj.weight")).reshape(B, -1, nh, hd)
    q = te_rmsnorm(q, _w(sd, p + "cross_attn.q_norm.weight"))
    k = te_rmsnorm(k, _w(sd, p + "cross_attn.k_norm.weight"))
    nv = ctx.shape[1] // 512
    if n_views > 1 and nv > 1:
        # MultiViewCrossAttention (multiview_dit.py:46-55): B (V L) D -> (V B) L D, context B (V M) D -> (V B) M D
        Lq = q.shape[1] // nv
        q = q.view(B, nv, Lq, nh, hd).transpose(0, 1).reshape(nv * B, Lq, nh, hd)
        k = k.view(B, nv, 512, nh, hd).transpose(0, 1).reshape(nv * B, 512, nh, hd)
        v = v.view(B, nv, 512, nh, hd).transpose(0, 1).reshape(nv * B, 512, nh, hd)
        o = sdpa(q, k, v).view(nv, B, Lq, nh * hd).transpose(0, 1).reshape(B, nv * Lq, nh * hd)
    else:
        o = sdpa(q, k, v)
    o = _lin(o, _w(sd, p + "cross_attn.output_proj.weight")).reshape(B, T, H, W, D)
    x = o * g_ca + x

    # MLP
    h = ln_mod(x, sh_ml, sc_ml)
    u = F.gelu(_lin(h, _w(sd, p + "mlp.layer1.weight")))
    y = _lin(u, _w(sd, p + "mlp.layer2.weight"))
    return x + g_ml * y


def dit_forward(cfg: dict, sd: dict, x_B_C_T_H_W: torch.Tensor, timesteps_B_T: torch.Tensor,
                crossattn_emb: torch.Tensor, cond_mask_B_1_T_H_W: torch.Tensor,
                padding_mask_B_1_H_W: torch.Tensor | None = None, action: torch.Tensor | None = None,
                view_ids=None) -> torch.Tensor:
    """-> velocity [B, C, T, H, W] fp32 (the model applies .float(), text2world_model_rectified_flow.py:860)."""
    x = x_B_C_T_H_W.to(act_dtype())
    B, C, T, Hl, Wl = x.shape
    x = torch.cat([x, cond_mask_B_1_T_H_W.to(act_dtype())], dim=1)  # minimal_v1_lvg_dit.py:46
    if not cfg.get("use_wan_fp32_strategy", True):
        # timesteps in the net dtype (module docstring); the fp32 truth takes the same bf16 input values
        t = timesteps_B_T.to(BF16)
        t = t * cfg["timestep_scale"] if act_dtype() == BF16 else t.float() * cfg["timestep_scale"]
    else:
        t = timesteps_B_T * cfg["timestep_scale"]
    if cfg["concat_padding_mask"]:
        pm = padding_mask_B_1_H_W if padding_mask_B_1_H_W is not None else torch.zeros(B, 1, Hl, Wl, device=x.device)
        pm = F.interpolate(pm.float(), size=(Hl, Wl), mode="nearest").to(act_dtype())
        x = torch.cat([x, pm[:, :, None].expand(B, 1, T, Hl, Wl)], dim=1)
    n_views = T // cfg["state_t"] if cfg.get("n_cameras_emb", 0) else 1
    if view_ids is None:
        view_ids = list(range(n_views))
    view_ids = [min(int(v), cfg.get("n_cameras_emb", 1) - 1) for v in view_ids]
    if cfg.get("view_condition_dim", 0):
        # concat_view_embedding (multiview_dit.py:462-490): view channels after [x, mask, padding mask]
        vidx = torch.tensor(view_ids, device=x.device)
        ve = _w(sd, "view_embeddings.weight")[vidx]  # [V, vdim] bf16
        Tv = T // n_views
        vch = ve.t()[None, :, :, None, None, None].expand(B, ve.shape[1], n_views, Tv, Hl, Wl)
        x = torch.cat([x.view(B, x.shape[1], n_views, Tv, Hl, Wl), vch.to(act_dtype())], 1).reshape(B, -1, T, Hl, Wl)
    ps, pt = cfg["patch_spatial"], cfg["patch_temporal"]
    Tp, Hp, Wp = T // pt, Hl // ps, Wl // ps
    # b c (t r) (h m) (w n) -> b t h w (c r m n)
    xp = x.reshape(B, x.shape[1], Tp, pt, Hp, ps, Wp, ps).permute(0, 2, 4, 6, 1, 3, 5, 7)
    xp = xp.reshape(B, Tp, Hp, Wp, -1)
    x = _lin(xp, _w(sd, "x_embedder.proj.1.weight"))
    # MultiCameraVideoRopePosition3DEmb (multiview_dit.py:108-130): positions restart per view
    freqs = rope_freqs(cfg, Tp // n_views, Hp, Wp, x.device).repeat(n_views, 1)

    ctx = crossattn_emb.to(act_dtype())
    if cfg["use_crossattn_projection"]:
        ctx = F.gelu(_lin(ctx, _w(sd, "crossattn_proj.0.weight"), _w(sd, "crossattn_proj.0.bias")))

    emb, lora = timestep_embedding(cfg, sd, t, action)
    view_mod = None
    if cfg.get("adaln_view_embedding"):
        # adaln_view_proj(adaln_view_embedder(view id)) (multiview_cross_dit.py:829-835, in cond_dtype) -> 9 chunks,
        # each per frame of its view, cast to the activation dtype
        cd = cond_dtype(cfg)
        e = _w(sd, "adaln_view_embedder.weight")[torch.tensor(view_ids, device=x.device)].to(cd)
        vp = _lin(e, _w(sd, "adaln_view_proj.weight").to(cd), _w(sd, "adaln_view_proj.bias").to(cd))
        view_mod = vp.to(act_dtype()).view(n_views, 9, -1).repeat_interleave(Tp // n_views, dim=0).transpose(0, 1)
    for i in range(cfg["num_blocks"]):
        x = block_forward(cfg, sd, i, x, emb, lora, ctx, freqs, n_views, view_mod, view_ids)

    # final layer (fp32 autocast, or bf16 ops without the fp32 strategy)
    D = cfg["model_channels"]
    cd = cond_dtype(cfg)
    sh, sc = adaln(sd, "final_layer.adaln_modulation", emb, lora[..., : 2 * D], n_chunks=2)
    xf = F.layer_norm(x.to(cd), (D,), eps=1e-6)
    xf = xf * (1 + sc[:, :, None, None, :]) + sh[:, :, None, None, :]
    out = _lin(xf, _w(sd, "final_layer.linear.weight").to(cd))  # [B,Tp,Hp,Wp, p1*p2*pt*C]
    Cout = cfg["out_channels"]
    out = out.reshape(B, Tp, Hp, Wp, ps, ps, pt, Cout).permute(0, 7, 1, 6, 2, 4, 3, 5)
    return out.reshape(B, Cout, Tp * pt, Hp * ps, Wp * ps).float()
