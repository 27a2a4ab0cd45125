"""fp8 linear layers (config 5's "fp8 MFMA" option): row quantisation kernels and the DiT's fp8 path.

The reference has no fp8 inference path, so nothing here is pinned to a reference output:
  * cp25_quant_fp8_rows is checked BIT-EXACT against the same definition in torch (scale = max|row| /
    448 in fp32, q = e4m3fn(clamp(x * (448 / max|row|))), RNE); cp25_gelu_quant_fp8 (fast erfc GELU)
    against that definition over cp25_gelu's exact-erf output: scales within a bf16 ulp, every code
    within one e4m3 step, >= 97 % of codes identical;
  * one fp8 projection vs fp32 math over the dequantised operands (q * s)(w8 * ws)^T: rel-L2 <= 4e-3
    (fp32 accumulation, one bf16 output rounding) -- checks the scale orientation end to end;
  * cp25_ln_mod_fp8 (LN-mod emitting the fp8 operand) bit-exact vs quant_fp8_rows(cp25_ln_mod);
  * a DiT forward with fp8 block GEMMs vs the bf16-path oracle: rel-L2 <= 6e-2 (stated precision cost
    of e4m3's 3 mantissa bits: ~3.7e-2 per GEMM on random operands; measured value printed).
"""
import dataclasses

import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

F8 = torch.float8_e4m3fn
FMAX = 448.0


def quant_ref(x: torch.Tensor):
    xf = x.float()
    amax = xf.abs().amax(dim=1, keepdim=True)
    inv = torch.where(amax > 0, torch.tensor(FMAX, device=x.device) / amax, torch.zeros_like(amax))
    q = (xf * inv).clamp(-FMAX, FMAX).to(F8)
    # tensor / tensor: IEEE division (torch turns `/ python_scalar` into a multiply by the reciprocal)
    return q, amax / torch.full_like(amax, FMAX)


@pytest.mark.parametrize("M,K", [(37, 512), (5, 2048), (33, 5120), (9, 8192), (3, 20480), (64, 3072)])
@pytest.mark.parametrize("gelu", [False, True])
def test_quant_rows_bit_exact(device, M, K, gelu):
    g = torch.Generator().manual_seed(M * 7 + K)
    x = (torch.randn(M, K, generator=g) * torch.logspace(-3, 2, M).unsqueeze(1)).to(device, torch.bfloat16)
    x[1] = 0  # all-zero row: q = 0, scale 0
    q, s = N.quant_fp8_rows(x, gelu=gelu)
    xr = x.clone()
    if gelu:
        N.gelu_(xr)
    qr, sr = quant_ref(xr)
    assert q.dtype == F8 and s.shape == (M, 1)
    if not gelu:
        assert torch.equal(s, sr)
        assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8))
        return
    # GELU variant: its fast erfc GELU is within ~1 bf16 ulp of cp25_gelu's exact one, so the row max
    # (scale) may move by a bf16 ulp and a few codes by one fp8 step
    assert torch.allclose(s, sr, rtol=2 ** -7, atol=0)
    d = q.float() * s - qr.float() * sr
    step = (qr.float().abs() * sr).clamp_min(1e-30) * 2.0 ** -3 + sr * 2.0 ** -9  # one e4m3 step (+ subnormal floor)
    assert (d.abs() <= step * 1.01).all()
    same = (q.view(torch.uint8) == qr.view(torch.uint8)).float().mean().item()
    assert same >= 0.97, same
    assert not torch.equal(xr, x)  # the input is left untouched


def test_quant_rows_rejects_bad_shapes(device):
    with pytest.raises(ValueError):
        N.quant_fp8_rows(torch.zeros(4, 1000, device=device, dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        N.quant_fp8_rows(torch.zeros(4, 2048, device=device, dtype=torch.float32))


def test_fp8_linear_matches_dequantised_math(device):
    from cosmos_predict2.dit import MinimalV1LVGDiT
    from cosmos_predict2.net_config import tiny_dit

    net = MinimalV1LVGDiT(tiny_dit(), device=device)
    net.set_linear_precision("fp8")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1000, 2048, generator=g).to(device, torch.bfloat16)
    w = (torch.randn(512, 2048, generator=g) * 0.02).to(device, torch.bfloat16)
    for gelu in (False, True):
        y = net._linear(x.clone(), w, f"w{gelu}", gelu_in=gelu)
        q, s = N.quant_fp8_rows(x, gelu=gelu)
        w8, ws = net._fp8_weight(f"w{gelu}", w)
        ref = (q.float() * s) @ (w8.float() * ws.t()).t()
        e = ((y.float() - ref).norm() / ref.norm()).item()
        assert e <= 4e-3, e
        # and the fp8 GEMM stays close to the bf16 one (the precision cost itself)
        xb = x.clone()
        if gelu:
            N.gelu_(xb)
        e_bf = ((y.float() - F.linear(xb, w).float()).norm() / F.linear(xb, w).float().norm()).item()
        assert e_bf <= 6e-2, e_bf


def test_dit_forward_fp8_vs_oracle(device):
    from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict
    from cosmos_predict2.net_config import tiny_dit
    from oracle import dit as odit

    cfg = tiny_dit(num_blocks=2)
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=0, zero_adaln_out=False).items()}
    g = torch.Generator().manual_seed(0)
    T, H, W = 3, 16, 16
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = torch.zeros(1, 1, T, H, W)
    mask[:, :, :1] = 1
    t = torch.tensor([[0.1, 877.0, 877.0]])
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    ref = odit.dit_forward(dataclasses.asdict(cfg), sd, x, t, ctx, mask)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd)
    args = (x.to(device).to(torch.bfloat16), t.to(device), ctx.to(device))
    out_bf = net(*args, condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu()
    net.set_linear_precision("fp8")
    out8 = net(*args, condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu()
    e_bf = ((out_bf - ref).norm() / ref.norm()).item()
    e8 = ((out8 - ref).norm() / ref.norm()).item()
    print(f"dit forward rel-L2 vs oracle: bf16 {e_bf:.3e}, fp8 {e8:.3e}")
    assert torch.isfinite(out8).all()
    assert e8 <= 6e-2, e8
    assert e8 > e_bf  # the fp8 path really ran
    net.set_linear_precision("bf16")
    assert torch.equal(net(*args, condition_video_input_mask_B_C_T_H_W=mask.to(device)).cpu(), out_bf)


@pytest.mark.parametrize("D,with_res", [(2048, True), (512, False), (5120, True)])
def test_ln_mod_fp8_equals_quantised_ln_mod(device, D, with_res):
    """cp25_ln_mod_fp8 == cp25_quant_fp8_rows(cp25_ln_mod(...)) bit for bit, x_out unchanged."""
    n, B, T, hw = 70, 2, 3, 32
    g = torch.Generator().manual_seed(D)
    x = torch.randn(n, B, D, generator=g).to(device, torch.bfloat16)
    y = torch.randn(n, B, D, generator=g).to(device, torch.bfloat16) if with_res else None
    mods = (torch.randn(B, T, 3 * D, generator=g) * 0.5).to(device, torch.bfloat16)
    sh, sc, gt = mods[..., :D], mods[..., D:2 * D], mods[..., 2 * D:]
    kw = dict(n_tok=n, B=B, tok0=5, hw=hw, x_st=B * D, x_sb=D)
    if with_res:
        kw.update(y=y, gate=gt)
    xo1 = torch.empty_like(x) if with_res else None
    xo2 = torch.empty_like(x) if with_res else None
    h = N.ln_mod(x, sh, sc, x_out=xo1, **kw)
    q, s = N.ln_mod(x, sh, sc, x_out=xo2, fp8=True, **kw)
    qr, sr = N.quant_fp8_rows(h.view(n * B, D))
    assert torch.equal(s, sr)
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8))
    if with_res:
        assert torch.equal(xo1, xo2)


@pytest.mark.parametrize("Lq,Lk,n_split", [(300, 1000, None), (513, 9000, 3), (256, 64, None)])
def test_prescaled_attention_vs_fp32(device, Lq, Lk, n_split):
    """cp25_attn_fwd_prescaled (the fp8 option's self-attention): q arrives multiplied by
    scale * log2(e) (rounded to bf16 there), P = exp2(q k^T); vs fp32 softmax(q k^T / sqrt(d)) v on the
    unscaled q: rel-L2 <= 4e-3 (the P/O bf16 floor plus the q * c rounding)."""
    B, H, D = 2, 3, 128
    g = torch.Generator().manual_seed(Lq + Lk)

    def rms_rows(L):
        x = torch.randn(B, L, H, D, generator=g)
        return x / x.pow(2).mean(-1, keepdim=True).sqrt()  # |row| = sqrt(128), like the DiT's q/k norm

    q, k = rms_rows(Lq), rms_rows(Lk)
    v = torch.randn(B, Lk, H, D, generator=g)
    qb = kb = D ** 0.5 * 1.02
    c = D ** -0.5 * 1.4426950408889634
    qd, kd, vd = q.to(device, torch.bfloat16), k.to(device, torch.bfloat16), v.to(device, torch.bfloat16)
    ref = torch.softmax(torch.einsum("blhd,bmhd->bhlm", qd.float(), kd.float()) * D ** -0.5, -1)
    ref = torch.einsum("bhlm,bmhd->blhd", ref, vd.float())
    qs = (qd.float() * c).to(torch.bfloat16)
    out = N.attn_fwd(qs, kd, vd, norm_bounds=(qb * c, kb), prescaled=True, n_split=n_split)
    e = ((out.float() - ref).norm() / ref.norm()).item()
    assert e <= 4e-3, e
    # bound products over 60 run the fixed per-row shift (up to 80) or the online max (beyond): same answer
    for nb in ((70.0 / kb, kb), (200.0 / kb, kb), None):
        o2 = N.attn_fwd(qs, kd, vd, norm_bounds=nb, prescaled=True, n_split=n_split)
        assert ((o2.float() - ref).norm() / ref.norm()).item() <= 4e-3, nb
