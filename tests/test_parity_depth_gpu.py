"""Full-depth parity at BASELINE config 1 geometry, measured against an fp32 truth.

Config 1 (256x256x9 frames -> latent [16, 3, 32, 32], 768 tokens) at the real 2B network: all 28
blocks, D 2048, 16 heads, crossattn_proj 100352 -> 1024, AdaLN-LoRA 256; seeded weights with the
reference's init distributions (AdaLN output layers randomised so modulation is exercised).

Three distances on identical inputs (rel-L2 of the fp32 output):
  hip  vs truth : the MI355X path against the fp32 truth (oracle.dit.fp32_truth(): the same bf16
                  weights, every activation in fp32);
  ref  vs truth : the bf16 oracle (the reference's inference arithmetic, op for op) against the truth;
  hip  vs ref   : the MI355X path against the bf16 oracle.
The reference itself is a bf16 computation, so its own distance from the truth is the scale of any
bf16 implementation's error: the gate is that the HIP path is no further from the truth than the bf16
reference restatement is (times a small factor), and hip-vs-ref is bounded by the measured values.
The reference's only numeric DiT test (CP vs non-CP, rel-L2 < 5e-3,
_src/predict2/interactive/networks/dit_causal_test.py:200-201) is the model for a bf16-vs-bf16 bound.
Measured values are printed (pytest -s) and recorded in DESIGN.md §4.
"""
import dataclasses

import pytest
import torch

from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict
from cosmos_predict2.model import Video2WorldModelRectifiedFlow
from cosmos_predict2.net_config import DIT_2B, SamplerConfig
from oracle import dit as odit
from oracle import sampler as osamp

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.fixture(scope="module")
def net2b():
    cfg = DIT_2B
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=11, zero_adaln_out=False).items()}
    return cfg, sd


def _report(name, hip, ref, truth):
    d = dict(hip_truth=rel(hip, truth), ref_truth=rel(ref, truth), hip_ref=rel(hip, ref))
    print(f"{name}: hip-vs-truth {d['hip_truth']:.3e}  bf16ref-vs-truth {d['ref_truth']:.3e}  "
          f"hip-vs-bf16ref {d['hip_ref']:.3e}")
    return d


@pytest.mark.parametrize("exact_q", [False, True])
def test_full_depth_2b_forward(device, net2b, exact_q):
    """One 28-block forward at config-1 geometry (cond frame t 0.1, the others mid-trajectory); both
    self-attention query roundings (exact_q: q rounded where the reference rounds it; default: q * c
    rounded once, the prescaled kernel)."""
    cfg, sd = net2b
    g = torch.Generator().manual_seed(31)
    T, H, W = 3, 32, 32
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = torch.zeros(1, 1, T, H, W)
    mask[:, :, :1] = 1
    t = torch.tensor([[0.1, 877.0, 877.0]])
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    c = dataclasses.asdict(cfg)
    ref = odit.dit_forward(c, sd, x, t, ctx, mask)
    with odit.fp32_truth():
        truth = odit.dit_forward(c, sd, x, t, ctx, mask)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd)
    net.exact_q_rounding = exact_q
    hip = net(x.to(device).to(torch.bfloat16), t.to(device), ctx.to(device),
              condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu()
    d = _report(f"28-block 2B forward (config-1 geometry, exact_q={exact_q})", hip, ref, truth)
    # the same reference with the flash-class attention numerics (bf16 P for P.V, what the reference's FA3 / cuDNN /
    # FA2 dispatch computes; oracle.dit.flash_sdpa, parity unpinned): hip-ref like with like
    with odit.flash_sdpa():
        ref_f = odit.dit_forward(c, sd, x, t, ctx, mask)
    df = _report(f"28-block 2B forward vs the flash-class reference (exact_q={exact_q})", hip, ref_f, truth)
    print(f"exact_q={exact_q}: hip-ref {d['hip_ref']:.3e} (fp32-P reference), {df['hip_ref']:.3e} (flash-class)")
    assert df["hip_ref"] <= 1.2e-2, df
    assert torch.isfinite(hip).all()
    # measured (MI355X, round 2): hip-truth 1.162e-2, ref-truth 1.164e-2, hip-ref 8.81e-3
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 1.2e-2, d


def test_full_depth_2b_forward_fp8_modes(device, net2b):
    """Config 5's fp8 options at full depth (no reference counterpart: the cost is stated against the fp32
    truth next to the bf16 reference's own distance): block GEMMs fp8, self-attention Q K^T fp8, both."""
    cfg, sd = net2b
    g = torch.Generator().manual_seed(31)
    T, H, W = 3, 32, 32
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = torch.zeros(1, 1, T, H, W)
    mask[:, :, :1] = 1
    t = torch.tensor([[0.1, 877.0, 877.0]])
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    c = dataclasses.asdict(cfg)
    ref = odit.dit_forward(c, sd, x, t, ctx, mask)
    with odit.fp32_truth():
        truth = odit.dit_forward(c, sd, x, t, ctx, mask)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd)
    args = (x.to(device).to(torch.bfloat16), t.to(device), ctx.to(device))
    dist, outs = {}, {}
    modes = (("bf16", "bf16"), ("bf16", "fp8qk"), ("bf16", "fp8"), ("fp8", "bf16"), ("fp8", "fp8"))
    for lin, att in modes:
        net.set_linear_precision(lin)
        net.set_attention_precision(att)
        outs[(lin, att)] = hip = net(*args, condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu()
        assert torch.isfinite(hip).all()
        dist[(lin, att)] = _report(f"28-block 2B forward, linear {lin}, attention {att}", hip, ref, truth)
    net.set_linear_precision("bf16")
    net.set_attention_precision("bf16")
    # measured (MI355X, round 2): hip-truth bf16/bf16 1.162e-2, bf16/fp8qk 1.171e-2, fp8/bf16 6.58e-2 (bf16
    # reference 1.164e-2): the fp8 Q K^T passes the bf16 path's own gate; the CPU emulation of the fp8 P.V
    # (tools/sim_fp8_attention_depth.py) put bf16/fp8 at 1.198e-2
    for att in ("fp8qk", "fp8"):
        assert not torch.equal(outs[("bf16", att)], outs[("bf16", "bf16")])  # the fp8 attention really ran
    assert dist[("bf16", "fp8qk")]["hip_truth"] <= 1.1 * dist[("bf16", "fp8qk")]["ref_truth"], dist
    assert dist[("bf16", "fp8")]["hip_truth"] <= 1.2 * dist[("bf16", "fp8")]["ref_truth"], dist
    for key in (("fp8", "bf16"), ("fp8", "fp8")):
        assert dist[key]["hip_truth"] <= 7e-2, dist


def test_full_depth_2b_forward_trained_size_norm_weights(device, net2b):
    """The 28-block forward with every q/k RMSNorm weight uniform in [0.5, 3] (trained-checkpoint scale, SURVEY A14;
    minimal_v4_dit.py:355-358): the weight bound product is ~150 log2 units, past the fixed-shift range, so every
    self- and cross-attention runs the online-max form (the report names it). Same truth gate as the unit weights."""
    cfg, sd0 = net2b
    g = torch.Generator().manual_seed(41)
    sd = dict(sd0)
    for k in sd:
        if k.endswith(("q_norm.weight", "k_norm.weight")):
            sd[k] = (0.5 + 2.5 * torch.rand(sd[k].shape, generator=g)).to(torch.bfloat16)
    T, H, W = 3, 32, 32
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = torch.zeros(1, 1, T, H, W)
    mask[:, :, :1] = 1
    t = torch.tensor([[0.1, 877.0, 877.0]])
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    c = dataclasses.asdict(cfg)
    ref = odit.dit_forward(c, sd, x, t, ctx, mask)
    with odit.fp32_truth():
        truth = odit.dit_forward(c, sd, x, t, ctx, mask)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd)
    kern = net.attention_kernels(T * H * W // 4)
    print("attention kernels:", kern)
    assert "online" in kern["self"] and "online" in kern["cross"], kern
    hip = net(x.to(device).to(torch.bfloat16), t.to(device), ctx.to(device),
              condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu()
    d = _report("28-block 2B forward, q/k norm weights in [0.5, 3]", hip, ref, truth)
    assert torch.isfinite(hip).all()
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 2e-2, d


@pytest.mark.parametrize("guidance", [0.0, 7.0])
def test_full_depth_2b_sampler(device, net2b, guidance):
    """Karras 2 steps (3 evaluations x CFG) of the 28-block 2B net at config-1 geometry, the metric's guidance 7 and
    guidance 0. The uncond branch gets the reference's context for is_negative_prompt=False: a zeroed embedding
    (TextAttr dropout, video2world_model_rectified_flow.py:167-170; model.py begin_sampling_from_batch), so c and u
    differ as they do in the metric run and c + 7 (c - u) does not amplify rounding noise ~15x the way two random
    contexts (c ~ u) would."""
    cfg, sd = net2b
    T, H, W = 3, 32, 32
    g = torch.Generator().manual_seed(71)
    gt = torch.randn(1, 16, T, H, W, generator=g)
    ctx_c = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    ctx_u = torch.zeros_like(ctx_c)
    c = dataclasses.asdict(cfg)
    kw = dict(num_cond=1, guidance=guidance, seed=0, num_steps=2, use_karras=True, cond_frame_t=0.1)
    ref = osamp.generate(c, sd, gt, ctx_c, ctx_u, **kw)
    with odit.fp32_truth():
        truth = osamp.generate(c, sd, gt, ctx_c, ctx_u, **kw)
    model = Video2WorldModelRectifiedFlow(cfg, SamplerConfig(use_kerras_sigma_at_inference=True,
                                                             conditional_frame_timestep=0.1), device=device)
    model.load_state_dict(sd)
    hip = model.sample_latents(gt.to(device), ctx_c.to(device), ctx_u.to(device), state_shape=(16, T, H, W),
                               num_conditional_frames=1, guidance=guidance, seed=0, num_steps=2).cpu()
    d = _report(f"28-block 2B sampler, Karras 2 steps, g={guidance}", hip, ref, truth)
    assert torch.isfinite(hip).all()
    # measured (MI355X, round 2, random uncond context): g=0 hip-truth 1.567e-2, ref-truth 1.563e-2, hip-ref
    # 1.274e-2; g=7 1.421e-1, 1.425e-1, 1.376e-1 (c ~ u: 7 (c - u) amplified the per-branch bf16 error ~15x)
    # measured (MI355X, round 3, zero uncond context): g=7 hip-truth 1.317e-1, ref-truth 1.300e-1, hip-ref 1.179e-1:
    # with random weights the text context barely moves the output, so c - u stays small even against a zeroed
    # uncond and 7 (c - u) still amplifies every per-branch rounding; the gates are therefore relative to the bf16
    # reference's own distance from exact math, which is the scale of that amplification
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= (1.6e-2 if guidance == 0 else 1.2 * d["ref_truth"]), d
    # regression gates (round 4, VERDICT r3: the gates above cannot see a few-percent regression): the measured ratios
    # with ~4 % margin -- g=0 hip-truth / ref-truth 1.001; g=7 1.013 and hip-ref / ref-truth 0.907
    assert d["hip_truth"] <= 1.05 * d["ref_truth"], d
    if guidance > 0:
        assert d["hip_ref"] <= 0.95 * d["ref_truth"], d


def test_full_depth_crossview_forward(device):
    """The 28-block 2B cross-view net (DIT_2B_MULTIVIEW_CROSSVIEW, multiview_cross_dit.py) against the fp32 truth:
    3 rig views (ids 0, 1, 5: front_wide with two of its three neighbours present, cross_right and cross_left with
    front_wide), 2 latent frames per view of 8 x 8 tokens, the same gate as the single-view forward."""
    from cosmos_predict2.net_config import DIT_2B_MULTIVIEW_CROSSVIEW

    cfg = DIT_2B_MULTIVIEW_CROSSVIEW.replace(state_t=2)
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=13, zero_adaln_out=False).items()}
    view_ids = [0, 1, 5]
    g = torch.Generator().manual_seed(37)
    T, H, W = 6, 16, 16
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = torch.zeros(1, 1, T, H, W)
    mask[:, :, ::2] = 1
    t = torch.tensor([[0.1, 877.0] * 3])
    ctx = torch.randn(1, 512 * 3, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    c = dataclasses.asdict(cfg)
    ref = odit.dit_forward(c, sd, x, t, ctx, mask, view_ids=view_ids)
    with odit.fp32_truth():
        truth = odit.dit_forward(c, sd, x, t, ctx, mask, view_ids=view_ids)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd)
    vi = torch.tensor([view_ids]).repeat_interleave(2, dim=1)
    hip = net(x.to(device).to(torch.bfloat16), t.to(device), ctx.to(device),
              condition_video_input_mask_B_C_T_H_W=mask.to(device), view_indices_B_T=vi.to(device)).cpu()
    d = _report("28-block 2B cross-view forward (3 views)", hip, ref, truth)
    assert torch.isfinite(hip).all()
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 1.2e-2, d
