"""BASELINE configs 3 and 4 at the network level, and the CP = 8 rank of config 3, on one MI355X.

* Config 3 (Predict2.5-14B: D 5120, 40 heads, 36 blocks, configs/video2world/defaults/net.py:58-94):
  (a) the full 36-block forward at config-1 geometry (latent [16, 3, 32, 32], 768 tokens) against the bf16 oracle and
      its fp32 truth, gated like the 2B (HIP no further from the truth than the bf16 reference x 1.1);
  (b) one CP = 8 rank at 720p x 121f: 13 640 local tokens of the 109 120, its self-attention reading the K/V of all
      109 120 tokens (captured from the CP = 1 forward, which is what the RCCL all-gather delivers); the rank's output
      rows must equal the same rows of the CP = 1 forward bit for bit (no key split: every row sees the same keys in
      the same order, and every projection is the hand-written GEMM, whose rows do not depend on M).
  (d) Video2World semantics (config 3 is V2W on the pre-trained 14B): 2 conditional latent frames, no
      conditional-frame timestep (one t for every frame), the shift-5 linspace schedule: the 36-block forward and a
      2-step CFG sampler (guidance 7, zeroed uncond context) against the oracle with the fp32-truth gate
      (video2world_model_rectified_flow.py:93-136; cosmos_predict2/config.py:459-469 for the frame counts).
* Config 4 (2B multiview, 7 views x 480p x 57 frames): multiview's "480p" is 480 x 832
  (predict2_multiview/configs/vid2vid/defaults/dataloader.py:163-168; the 16:9 bucket of predict2/datasets/utils.py:32),
  so 7 x 15 latent frames of 30 x 52 patches = 163 800 tokens, joint self-attention over all views, per-view text
  cross-attention (predict2_multiview/networks/multiview_dit.py):
  (c) the 28-block forward at that geometry (finite), and a one-block forward at that geometry against the oracle.
The oracle is the CPU restatement (oracle/dit.py); at these sizes it runs on the GPU's own torch ops (fp32
matmuls, hipBLASLt bf16 GEMMs with fp32 accumulation), never on this repository's kernels (hours on host cores).
"""
import dataclasses

import pytest
import torch

from cosmos_predict2 import _native as N
from cosmos_predict2 import context_parallel as cpx
from cosmos_predict2 import dit as dit_mod
from cosmos_predict2.dit import Geometry, MinimalV1LVGDiT, init_state_dict
from cosmos_predict2.model import Video2WorldModelRectifiedFlow
from cosmos_predict2.net_config import DIT_14B, DIT_2B_MULTIVIEW, SAMPLER_PRE_TRAINED
from oracle import dit as odit
from oracle import sampler as osamp

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def _report(name, hip, ref, truth=None):
    d = dict(hip_ref=rel(hip, ref))
    if truth is not None:
        d.update(hip_truth=rel(hip, truth), ref_truth=rel(ref, truth))
    print(f"{name}: " + "  ".join(f"{k} {v:.3e}" for k, v in d.items()))
    return d


@pytest.fixture(scope="module")
def sd14(device):
    """Seeded 14B weights with the reference's init distributions (AdaLN output layers randomised), made on the GPU."""
    sd = init_state_dict(DIT_14B, seed=13, device=device, zero_adaln_out=False)
    yield {"net." + k: v for k, v in sd.items()}
    del sd
    torch.cuda.empty_cache()


def test_config3_14b_full_depth_vs_oracle(device, sd14):
    cfg = DIT_14B
    g = torch.Generator().manual_seed(31)
    T, H, W = 3, 32, 32
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = torch.zeros(1, 1, T, H, W)
    mask[:, :, :1] = 1
    t = torch.tensor([[0.1, 877.0, 877.0]])
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(BF16)
    c = dataclasses.asdict(cfg)
    args = (x.to(device), t.to(device), ctx.to(device), mask.to(device))
    with torch.no_grad():
        ref = odit.dit_forward(c, sd14, *args).cpu()
        with odit.fp32_truth():
            truth = odit.dit_forward(c, sd14, *args).cpu()
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd14)
    hip = net(x.to(device).to(BF16), t.to(device), ctx.to(device), condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu()
    del net
    torch.cuda.empty_cache()
    d = _report("14B 36-block forward (config-1 geometry)", hip, ref, truth)
    assert torch.isfinite(hip).all()
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 1.5e-2, d


def test_config3_cp8_rank_matches_cp1_rows(device, sd14, monkeypatch):
    cfg = DIT_14B
    T, Hp, Wp = 31, 44, 80
    L, world = T * Hp * Wp, 8
    n = L // world
    D = cfg.model_channels
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd14)
    g = torch.Generator(device=device).manual_seed(5)
    rows = torch.randn(L, 1, 72, device=device, generator=g).to(BF16)
    t_B_T = torch.full((1, T), 0.5, device=device)
    t_B_T[0, 0] = 0.0001
    ctx = net.prepare_context(torch.randn(1, 512, cfg.crossattn_proj_in_channels, device=device, generator=g).to(BF16))
    monkeypatch.setattr(N, "_ATTN_SPLIT", 1)
    # CP = 1, capturing every self-attention's K and V (what the rank's all-gather returns)
    kv_blocks = []
    orig_attn = N.attn_fwd

    def capture(q, k, v, *a, **kw):
        if k.shape[1] == L:
            kv = torch.empty((L, 2, D), dtype=BF16, device=device)
            kv[:, 0].copy_(k[0].reshape(L, D))
            kv[:, 1].copy_(v[0].reshape(L, D))
            kv_blocks.append(kv)
        return orig_attn(q, k, v, *a, **kw)

    monkeypatch.setattr(N, "attn_fwd", capture)
    with torch.no_grad():
        ref = net.forward_tokens(rows, t_B_T, ctx, Geometry(T=T, Hp=Hp, Wp=Wp, tok0=0, n_tok=L))
    monkeypatch.setattr(N, "attn_fwd", orig_attn)
    assert len(kv_blocks) == cfg.num_blocks
    # a CP = 8 rank: the K/V all-gather delivers the full K|V rows of each block
    calls = []

    def gather(out, x, group):
        out.view(L, 2 * D).copy_(kv_blocks[len(calls)].view(L, 2 * D))
        calls.append(x.shape[0])
        return cpx._Done()

    monkeypatch.setattr(dit_mod, "all_gather_into_async", gather)
    monkeypatch.setattr(torch.distributed, "get_world_size", lambda group=None: world)
    net.cp_group = object()
    try:
        for r in (3, 7):  # rank 3's range starts inside frame 11; rank 7 is the last
            calls.clear()
            geo = Geometry(T=T, Hp=Hp, Wp=Wp, tok0=r * n, n_tok=n)
            with torch.no_grad():
                out = net.forward_tokens(rows[r * n:(r + 1) * n], t_B_T, ctx, geo)
            assert calls == [n] * cfg.num_blocks  # every block gathered this rank's n K/V rows
            exp = ref[r * n:(r + 1) * n]
            same = (out == exp).float().mean().item()
            print(f"14B CP=8 rank {r} ({n} tokens from {r * n}): bit-identical fraction {same:.6f}, "
                  f"rel-L2 {rel(out, exp):.2e}")
            assert torch.isfinite(out).all()
            assert torch.equal(out, exp)
    finally:
        net.cp_group = None
    del net, kv_blocks
    torch.cuda.empty_cache()


def test_config3_v2w_14b_forward_two_cond_frames(device, sd14):
    """Video2World conditioning on the 14B: latent frames 0 and 1 conditioned (mask and ground-truth frames), one t for
    every frame (conditional_frame_timestep off: the pre-trained sampler config), 36 blocks."""
    cfg = DIT_14B
    g = torch.Generator().manual_seed(37)
    T, H, W = 3, 32, 32
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = osamp.frame_mask(1, T, H, W, 2)
    t = torch.tensor([[613.0]])  # [B, 1]: the same t for every frame, conditional ones included
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(BF16)
    c = dataclasses.asdict(cfg)
    args = (x.to(device), t.to(device), ctx.to(device), mask.to(device))
    with torch.no_grad():
        ref = odit.dit_forward(c, sd14, *args).cpu()
        with odit.fp32_truth():
            truth = odit.dit_forward(c, sd14, *args).cpu()
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd14)
    hip = net(x.to(device).to(BF16), t.to(device), ctx.to(device), condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu()
    del net
    torch.cuda.empty_cache()
    d = _report("14B V2W forward (2 cond frames, no cond timestep)", hip, ref, truth)
    assert torch.isfinite(hip).all()
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 1.5e-2, d


def test_config3_v2w_14b_sampler(device, sd14):
    """Two UniPC steps of the 14B Video2World sampler as config 3 runs it (SAMPLER_PRE_TRAINED: shift-5 linspace schedule,
    no Karras sigmas, no conditional-frame timestep), 2 conditional latent frames (frame replacement and the ground-
    truth velocity on both), guidance 7 against a zeroed uncond context, vs the oracle loop and its fp32 truth."""
    cfg = DIT_14B
    scfg = SAMPLER_PRE_TRAINED
    assert scfg.conditional_frame_timestep < 0 and not scfg.use_kerras_sigma_at_inference
    T, H, W = 3, 32, 32
    g = torch.Generator().manual_seed(73)
    gt = torch.randn(1, 16, T, H, W, generator=g)
    ctx_c = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(BF16)
    ctx_u = torch.zeros_like(ctx_c)
    c = dataclasses.asdict(cfg)
    kw = dict(num_cond=2, guidance=7.0, seed=1, num_steps=2, shift=5.0, use_karras=False, cond_frame_t=-1.0)
    dv = [a.to(device) for a in (gt, ctx_c, ctx_u)]
    with torch.no_grad():
        ref = osamp.generate(c, sd14, *dv, **kw).cpu()
        with odit.fp32_truth():
            truth = osamp.generate(c, sd14, *dv, **kw).cpu()
    model = Video2WorldModelRectifiedFlow(cfg, scfg, device=device)
    model.load_state_dict(sd14)
    hip = model.sample_latents(*dv, state_shape=(16, T, H, W), num_conditional_frames=2, guidance=7.0, seed=1,
                               num_steps=2, shift=5.0).cpu()
    del model
    torch.cuda.empty_cache()
    d = _report("14B V2W sampler, shift 5, 2 steps, 2 cond frames, g=7", hip, ref, truth)
    assert torch.isfinite(hip).all()
    # the conditional frames leave the sampler as the ground truth (velocity replaced by noise - gt on them)
    cond_err = rel(hip[:, :, :2], ref[:, :, :2])
    print(f"  conditional frames vs oracle: rel-L2 {cond_err:.3e}")
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 1.2 * d["ref_truth"], d
    # regression gates from the measured ratios (MI355X, round 4: hip-truth / ref-truth 0.998, hip-ref / ref-truth 0.814)
    assert d["hip_truth"] <= 1.05 * d["ref_truth"], d
    assert d["hip_ref"] <= 0.9 * d["ref_truth"], d


def _mv_inputs(cfg, V, Tv, Hl, Wl, seed, device):
    g = torch.Generator(device=device).manual_seed(seed)
    T = V * Tv
    x = torch.randn(2, 16, T, Hl, Wl, device=device, generator=g)
    mask = torch.zeros(2, 1, T, Hl, Wl, device=device)
    for v in range(V):
        mask[:, :, v * Tv] = 1.0  # the first frame of every view conditions
    t = torch.full((2, T), 500.0, device=device)
    t[:, ::Tv] = 0.1
    ctx = torch.randn(2, 512 * V, cfg.crossattn_proj_in_channels, device=device, generator=g).to(BF16)
    return x, t, ctx, mask


def test_config4_multiview_7view_480p(device):
    V, Tv, Hl, Wl = 7, 15, 60, 104  # 57 frames at 480 x 832 per view -> 15 latent frames of 30 x 52 patches
    cfg = DIT_2B_MULTIVIEW.replace(state_t=Tv)
    L = V * Tv * (Hl // 2) * (Wl // 2)
    assert L == 163800  # not a multiple of 64 or 256: ragged last key tile and query block
    # the full 28-block forward (CFG pair as B = 2)
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=17, device=device, zero_adaln_out=False).items()}
    x, t, ctx, mask = _mv_inputs(cfg, V, Tv, Hl, Wl, 18, device)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd)
    assert net.n_views_for(V * Tv) == V
    with torch.no_grad():
        out = net(x.to(BF16), t, ctx, condition_video_input_mask_B_C_T_H_W=mask)
    torch.cuda.synchronize()
    print(f"config 4 28-block forward: {L} tokens, out {tuple(out.shape)}, |out| {out.float().norm():.3e}")
    assert out.shape == (2, 16, V * Tv, Hl, Wl)
    assert torch.isfinite(out).all()
    del out, net
    # one block at the same geometry against the oracle (joint attention over all 136 080 tokens, per-view text
    # cross-attention), on every output row and on the block-0 query slice of each view's first frame
    cfg1 = cfg.replace(num_blocks=1)
    sd1 = {k: v for k, v in sd.items() if not k.startswith("net.blocks.") or k.startswith("net.blocks.0.")}
    net1 = MinimalV1LVGDiT(cfg1, device=device)
    net1.load_state_dict(sd1)
    with torch.no_grad():
        hip = net1(x.to(BF16), t, ctx, condition_video_input_mask_B_C_T_H_W=mask)
        ref = odit.dit_forward(dataclasses.asdict(cfg1), sd1, x, t, ctx, mask)
    d = _report("config 4 one-block forward (163 800 tokens, 7 views)", hip, ref)
    first = hip[:, :, ::Tv], ref[:, :, ::Tv]
    e_first = rel(*first)
    print(f"  first frame of every view: rel-L2 {e_first:.3e}")
    assert torch.isfinite(hip).all()
    assert d["hip_ref"] <= 1e-2, d
    assert e_first <= 1e-2, e_first
