"""Per-op distance table: every HIP op of the hot path against the reference's own bf16 op sequence (the oracle's
functions, run with torch on the same device and inputs) and against fp32 math, at the 2B widths.

This is the table DESIGN.md §4 quotes for the north star's "1e-3 rel-L2 of the reference": for each op it records
rel-L2(HIP, bf16 reference), rel-L2(HIP, fp32) and rel-L2(bf16 reference, fp32), and whether the first is <= 1e-3.
Ops whose last step is one bf16 rounding of the same fp32 value land at 0 or a few 1e-4 (an occasional one-ulp flip);
ops that round intermediates at different points than the reference (attention's P and O, the GEMM's accumulation
order) sit at the bf16 noise floor, about 1e-3 to 3e-3, on both sides of the truth equally. The asserted bounds are
each op's tolerance from its own test file; the 1e-3 column is reported, not asserted.
The table is written to gpurun_out/op_table.json when that directory exists (GPU box runs).
"""
import json
import math
import os

import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N
from cosmos_predict2.vae import _Conv
from oracle import dit as odit
from oracle import vae as ovae

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16
TABLE = {}
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


def record(op, hip, ref, truth, bound, note=""):
    row = dict(hip_ref=rel(hip, ref), hip_truth=rel(hip, truth), ref_truth=rel(ref, truth))
    row["meets_1e-3"] = row["hip_ref"] <= 1e-3
    row["bound"] = bound
    if note:
        row["note"] = note
    TABLE[op] = row
    print(f"{op}: hip-ref {row['hip_ref']:.2e}  hip-truth {row['hip_truth']:.2e}  ref-truth {row['ref_truth']:.2e}")
    assert torch.isfinite(hip.float()).all()
    assert row["hip_ref"] <= bound, row
    return row


@pytest.fixture(scope="module", autouse=True)
def _dump():
    yield
    out = os.path.join(ROOT, "gpurun_out")
    if TABLE and os.path.isdir(out):
        with open(os.path.join(out, "op_table.json"), "w") as f:
            json.dump(TABLE, f, indent=1)


def _mods(B, T, D, g, dev, s=0.5):
    m = (torch.randn(B, T, 3 * D, generator=g, device=dev) * s).to(BF16)
    return m[..., :D], m[..., D:2 * D], m[..., 2 * D:]


def test_ln_mod_gated_residual(device):
    """cp25_ln_mod: x' = x + g y, h = LN(x') (1 + scale) + shift (minimal_v4_dit.py:1171-1246)."""
    n, B, D, T, hw = 2048, 2, 2048, 4, 512
    g = torch.Generator(device=device).manual_seed(1)
    x = torch.randn(n, B, D, generator=g, device=device).to(BF16)
    y = torch.randn(n, B, D, generator=g, device=device).to(BF16)
    sh, sc, gt = _mods(B, T, D, g, device)
    x_out = torch.empty_like(x)
    h = N.ln_mod(x, sh, sc, n_tok=n, B=B, tok0=0, hw=hw, x_st=B * D, x_sb=D, y=y, gate=gt, x_out=x_out)
    fr = torch.arange(n, device=device) // hw
    G, Sh, Sc = (t[:, fr].transpose(0, 1) for t in (gt, sh, sc))
    xr = x + G * y
    ref = odit.ln_mod(xr, Sh, Sc)
    xt = x.float() + G.float() * y.float()
    truth = F.layer_norm(xt, (D,), eps=1e-6) * (1 + Sc.float()) + Sh.float()
    record("gated residual x + g*y (cp25_ln_mod x_out)", x_out, xr, xt, 0.0)
    record("LN-mod (cp25_ln_mod h)", h, ref, truth, 2e-3)


def test_head_rmsnorm_rope(device):
    """cp25_head_rmsnorm_rope: TE RMSNorm (bf16 out) + RoPE in fp32, one bf16 rounding (minimal_v4_dit.py:411-419)."""
    n, B, H = 1024, 2, 16
    D = H * 128
    g = torch.Generator(device=device).manual_seed(2)
    buf = torch.randn(n * B, 3 * D, generator=g, device=device).to(BF16)
    w = (1 + 0.3 * torch.randn(128, generator=g, device=device)).to(BF16)
    fr = torch.rand(n, 64, generator=g, device=device) * 50
    src = buf[:, D:2 * D].clone().view(n, B, H, 128).transpose(0, 1)  # [B, n, H, 128]
    N.head_rmsnorm_rope(buf, n_rows=n * B, B=B, H=H, head_off=D, weight=w, cos=torch.cos(fr), sin=torch.sin(fr))
    hip = buf[:, D:2 * D].view(n, B, H, 128).transpose(0, 1)
    freqs = torch.cat([fr, fr], -1)
    ref = odit.apply_rope(odit.te_rmsnorm(src, w).float(), freqs).to(BF16)
    sf = src.float()
    truth = odit.apply_rope(sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + 1e-6) * w.float(), freqs)
    record("q/k RMSNorm + RoPE (cp25_head_rmsnorm_rope)", hip, ref, truth, 2e-3)


def _qkv(B, L, Lk, H, g, dev, wq=1.0, q_fp32=False):
    q = torch.randn(B, L, H, 128, generator=g, device=dev)
    k = torch.randn(B, Lk, H, 128, generator=g, device=dev)
    q32 = q * torch.rsqrt(q.pow(2).mean(-1, keepdim=True)) * wq  # the q RMSNorm's fp32 result before its bf16 rounding
    q = q32.to(BF16)
    k = (k * torch.rsqrt(k.pow(2).mean(-1, keepdim=True))).to(BF16)
    v = torch.randn(B, Lk, H, 128, generator=g, device=dev).to(BF16)
    return (q, k, v, q32) if q_fp32 else (q, k, v)


def _attn_truth(q, k, v, qf=None):
    qf = q.float() if qf is None else qf
    s = torch.einsum("blhd,bmhd->bhlm", qf, k.float()) * 128 ** -0.5
    return torch.einsum("bhlm,bmhd->blhd", torch.softmax(s, -1), v.float())


@pytest.mark.parametrize("Lk", [4096, 512])
def test_attention(device, Lk):
    """cp25_attn_fwd_* (networks/attention.py:90-181): both the form with q rounded where the reference rounds it
    (bounded) and the DiT's default (q * scale * log2 e rounded once, prescaled). The truth keeps q in fp32 (the q
    RMSNorm's result before any rounding): the reference rounds it to bf16 once, the DiT's prescaled form rounds q * c
    once (its RMSNorm/RoPE kernel emits bf16(q c) from fp32), so each path carries exactly one q rounding. (Rounding an
    already bf16 q times c again -- bf16(bf16(q) c), as this test did until round 4 -- adds a second rounding and read
    as a 21 % parity cost of the prescaled form that the DiT does not have: tests/test_prescaled_q_cpu.py.)"""
    B, L, H = 1, 4096, 4
    g = torch.Generator(device=device).manual_seed(3 + Lk)
    q, k, v, q32 = _qkv(B, L, Lk, H, g, device, q_fp32=True)
    ref = odit.sdpa(q, k, v).view(B, L, H, 128)
    truth = _attn_truth(q, k, v, qf=q32)
    bounds = (q.float().norm(dim=-1).max().item() * 1.01, k.float().norm(dim=-1).max().item() * 1.01)
    kind = "self" if Lk > 512 else "cross (Lk 512)"
    hip = N.attn_fwd(q, k, v, norm_bounds=bounds)
    record(f"{kind}-attention, q rounded as the reference (cp25_attn_fwd_bounded)", hip, ref, truth, 4e-3)
    c = 128 ** -0.5 * math.log2(math.e)
    qs = (q32 * c).to(BF16)
    hip_p = N.attn_fwd(qs, k, v, prescaled=True, norm_bounds=(bounds[0] * c * 1.01, bounds[1]))
    record(f"{kind}-attention, DiT default: q*c rounded once (cp25_attn_fwd_prescaled)", hip_p, ref, truth, 4e-3)
    # like with like: the reference's real kernels (flash / cuDNN SDPA) round P to bf16 for P.V as these kernels do;
    # the flash-class oracle (oracle.dit.flash_sdpa: FlashAttention-2's forward numerics, parity unpinned) is that
    # reference, so hip-ref here is the bf16-P floor between two flash-class implementations
    with odit.flash_sdpa():
        ref_f = odit.sdpa(q, k, v).view(B, L, H, 128)
    record(f"{kind}-attention vs flash-class reference (bf16 P), q rounded as the reference", hip, ref_f, truth, 4e-3,
           note="reference = oracle.dit.flash_sdpa (FlashAttention-2 Algorithm 1 numerics)")
    record(f"{kind}-attention vs flash-class reference (bf16 P), DiT default q*c", hip_p, ref_f, truth, 4e-3,
           note="reference = oracle.dit.flash_sdpa (FlashAttention-2 Algorithm 1 numerics)")


def test_block_gemms(device):
    """cp25_gemm_epi / cp25_gemm_res (minimal_v4_dit.py:227-254, 400-432, 1213-1244): projection, MLP1 + GELU, and the
    output projection with the gated residual, vs the bf16 linear (fp32 accumulation, one rounding) of the reference."""
    M, K, Nn, B, T, hw = 4096, 2048, 2048, 2, 4, 512
    g = torch.Generator(device=device).manual_seed(4)
    a = torch.randn(M, K, generator=g, device=device).to(BF16)
    w = (torch.randn(Nn, K, generator=g, device=device) * K ** -0.5).to(BF16)
    w1 = (torch.randn(4 * Nn, K, generator=g, device=device) * K ** -0.5).to(BF16)
    truth = a.float() @ w.float().t()
    ref = F.linear(a, w)
    record("projection GEMM (cp25_gemm_epi)", N.gemm_epi(a, w), ref, truth, 4e-3)
    t1 = a.float() @ w1.float().t()
    record("MLP layer1 + GELU epilogue (cp25_gemm_epi GELU)", N.gemm_epi(a, w1, epilogue=N.EPI_GELU),
           F.gelu(F.linear(a, w1)), F.gelu(t1), 4e-3)
    x = torch.randn(M // B, B, Nn, generator=g, device=device).to(BF16)
    _, _, gate = _mods(B, T, Nn, g, device)
    hip = N.gemm_res(a, w, x, B * Nn, Nn, gate, B=B, tok0=0, hw=hw).view(M // B, B, Nn)
    G = gate[:, torch.arange(M // B, device=device) // hw].transpose(0, 1)
    ref_r = x + G * ref.view(M // B, B, Nn)
    truth_r = x.float() + G.float() * truth.view(M // B, B, Nn)
    record("output projection + gated residual epilogue (cp25_gemm_res)", hip, ref_r, truth_r, 4e-3)


def test_gelu(device):
    x = (torch.randn(1 << 20, device=device) * 2).to(BF16)
    y = N.gelu_(x.clone())
    xd = x.double()
    truth = xd * 0.5 * torch.special.erfc(-xd * 0.5 ** 0.5)
    record("GELU (cp25_gelu)", y, F.gelu(x), truth, 2e-3, "torch's bf16 GELU cancels for x << 0; HIP uses erfc")


def test_final_ln_mod(device):
    n, B, D, T, hw = 1024, 2, 2048, 2, 512
    g = torch.Generator(device=device).manual_seed(5)
    x = torch.randn(n, B, D, generator=g, device=device).to(BF16)
    y = torch.randn(n, B, D, generator=g, device=device).to(BF16)
    _, _, gt = _mods(B, T, D, g, device, 1.0)
    sh, sc = torch.randn(B, T, 2 * D, generator=g, device=device).chunk(2, -1)
    out = N.final_ln_mod(x, sh, sc, n_tok=n, B=B, tok0=0, hw=hw, y=y, gate=gt)
    fr = torch.arange(n, device=device) // hw
    G, Sh, Sc = gt[:, fr].transpose(0, 1), sh[:, fr].transpose(0, 1), sc[:, fr].transpose(0, 1)
    xr = x + G * y
    ref = F.layer_norm(xr.float(), (D,), eps=1e-6) * (1 + Sc) + Sh
    truth = F.layer_norm(x.float() + G.float() * y.float(), (D,), eps=1e-6) * (1 + Sc) + Sh
    record("final layer LN-mod (cp25_final_ln_mod)", out, ref, truth, 1e-5)


def test_fp32_linears(device):
    """cp25_gemm_f32: the final layer's Linear(D, 64) over the tokens (minimal_v4_dit.py:993-995) and the AdaLN-LoRA
    second layer with its LoRA addend (:1136-1154), against the reference's fp32 F.linear (torch's fp32 GEMM on the
    same device; TF32 off) and float64."""
    g = torch.Generator(device=device).manual_seed(8)
    x = torch.randn(8192, 2048, generator=g, device=device)
    w = torch.randn(64, 2048, generator=g, device=device) * 2048 ** -0.5
    record("final linear fp32 (cp25_gemm_f32)", N.gemm_f32(x, w, split_k=False), F.linear(x, w),
           x.double() @ w.double().t(), 1e-5)
    a1 = torch.randn(62, 84 * 256, generator=g, device=device).view(62, 84, 256).transpose(0, 1)
    w2 = torch.randn(84, 6144, 256, generator=g, device=device) * 256 ** -0.5
    lora = torch.randn(62, 6144, generator=g, device=device)
    record("AdaLN-LoRA layer 2 + LoRA fp32 (cp25_gemm_f32, batched)", N.gemm_f32(a1, w2, add=lora),
           torch.bmm(a1, w2.transpose(1, 2)) + lora, torch.bmm(a1.double(), w2.double().transpose(1, 2)) + lora.double(),
           1e-5)


def test_layer_norm_affine(device):
    """cp25_layer_norm: the cross-view net's affine LayerNorm (multiview_cross_dit.py:290, :441) against torch's bf16
    F.layer_norm (the reference's op) and fp32."""
    g = torch.Generator(device=device).manual_seed(9)
    D = 2048
    x = (torch.randn(4096, D, generator=g, device=device) * 2 + 0.5).to(BF16)
    w = (1 + 0.2 * torch.randn(D, generator=g, device=device)).to(BF16)
    b = (0.2 * torch.randn(D, generator=g, device=device)).to(BF16)
    record("affine LayerNorm (cp25_layer_norm)", N.layer_norm(x, w, b), F.layer_norm(x, (D,), w, b, eps=1e-6),
           F.layer_norm(x.float(), (D,), w.float(), b.float(), eps=1e-6), 2e-3)


def test_vae_ops(device):
    """cp25_conv3d (CausalConv3d, wan2pt1.py:44-62), cp25_rms_norm_silu (RMS_norm + SiLU, :64-85),
    cp25_vae_attn (AttentionBlock core, :214-261)."""
    g = torch.Generator(device=device).manual_seed(6)
    C, H, W = 96, 32, 64
    x = torch.randn(1, C, 3, H, W, generator=g, device=device).to(BF16)
    w = (torch.randn(C, C, 3, 3, 3, generator=g, device=device) / (27 * C) ** 0.5).to(BF16)
    b = (0.1 * torch.randn(C, generator=g, device=device)).to(BF16)
    ref = ovae._conv3d(x, w, b, 1)  # 2 causal zero frames in front, fp32 conv, one rounding
    truth = F.conv3d(F.pad(x.float(), (1, 1, 1, 1, 2, 0)), w.float(), b.float())
    conv = _Conv(w, b, device)
    xl = x[0].permute(1, 2, 3, 0).contiguous()
    hip = conv([None, None, xl[0], xl[1], xl[2]], 3, H, W, pad=(1, 1, 1, 1)).permute(3, 0, 1, 2)[None]
    record("VAE causal 3x3x3 conv (cp25_conv3d halo)", hip, ref, truth, 2e-3)
    gam = (1 + 0.2 * torch.randn(C, generator=g, device=device)).to(BF16)
    xs = torch.randn(2, H, W, C, generator=g, device=device).to(BF16)
    hip = N.rms_norm_silu(xs, gam)
    ref = ovae.silu(ovae.rms_norm(xs, gam, channel_dim=-1))
    xf = xs.float()
    truth = F.silu(xf / xf.norm(dim=-1, keepdim=True) * C ** 0.5 * gam.float())
    record("VAE RMS_norm + SiLU (cp25_rms_norm_silu)", hip, ref, truth, 4e-3)
    L, D = 1024, 384
    q = torch.randn(1, L, D, generator=g, device=device).to(BF16)
    k = torch.randn(1, L, D, generator=g, device=device).to(BF16)
    v = torch.randn(1, L, D, generator=g, device=device).to(BF16)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * D ** -0.5
    truth = torch.matmul(torch.softmax(s, -1), v.float())
    hip = N.vae_attn(q, k, v)
    record("VAE attention core (cp25_vae_attn)", hip, truth.to(BF16), truth, 4e-3,
           "the reference computes this core in fp32 and rounds once")
