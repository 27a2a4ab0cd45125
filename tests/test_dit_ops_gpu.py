"""Parity of the DiT elementwise HIP kernels and the fused UniPC step.

Oracles: the reference's op sequences (bf16 torch ops, minimal_v4_dit.py:1171-1246; fp32 UniPC math,
fm_solvers_unipc.py) evaluated with torch on the same inputs.
Tolerances:
  * cp25_unipc_step, cp25_patchify, cp25_cfg_velocity: bit-exact (same IEEE fp32 op sequence);
  * LN-modulate / RMSNorm-RoPE / GELU: every element within 1 bf16 ulp of the oracle and >= 99.9 %
    of elements identical (the reference's LayerNorm / erf / cos come from other fp32 libraries,
    so a 1-ulp flip of the final bf16 rounding is possible).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N
from cosmos_predict2.scheduler import FlowUniPCMultistepScheduler
from oracle.unipc import UniPC

pytestmark = pytest.mark.gpu


def bf16_ulp_close(a, b, min_equal=0.999):
    a32, b32 = a.float(), b.float()
    eq = (a32 == b32).float().mean().item()
    # 1 ulp at bf16 = 2^-7 relative to the exponent of the larger magnitude
    ulp = torch.clamp(torch.maximum(a32.abs(), b32.abs()), min=1e-30)
    ulp = torch.pow(2.0, torch.floor(torch.log2(ulp)) - 7)
    ok = ((a32 - b32).abs() <= ulp * 1.0001).all().item()
    return eq >= min_equal and ok, eq


def test_ln_mod_with_residual(device):
    n, B, D, T, hw = 96, 2, 2048, 3, 32
    g = torch.Generator().manual_seed(0)
    x = torch.randn(n, B, D, generator=g).to(device, torch.bfloat16)
    y = torch.randn(n, B, D, generator=g).to(device, torch.bfloat16)
    mods = (torch.randn(B, T, 3 * D, generator=g) * 0.5).to(device, torch.bfloat16)
    sh, sc, gt = mods[..., :D], mods[..., D:2 * D], mods[..., 2 * D:]
    x_out = torch.empty_like(x)
    h = N.ln_mod(x, sh, sc, n_tok=n, B=B, tok0=0, hw=hw, x_st=B * D, x_sb=D, y=y, gate=gt, x_out=x_out)
    tok = torch.arange(n, device=device)
    fr = tok // hw
    G = gt[:, fr].transpose(0, 1)  # [n, B, D]
    Sh = sh[:, fr].transpose(0, 1)
    Sc = sc[:, fr].transpose(0, 1)
    xr = x + G * y
    assert torch.equal(x_out, xr)
    hr = F.layer_norm(xr, (D,), eps=1e-6) * (1 + Sc) + Sh
    ok, eq = bf16_ulp_close(h, hr)
    assert ok, eq


def test_ln_mod_broadcast_input(device):
    n, B, D, T, hw = 64, 2, 512, 3, 32  # tokens 32..95 span frames 1..2
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, 1, D, generator=g).to(device, torch.bfloat16)
    mods = (torch.randn(B, T, 3 * D, generator=g) * 0.5).to(device, torch.bfloat16)
    sh, sc = mods[..., :D], mods[..., D:2 * D]
    h = N.ln_mod(x, sh, sc, n_tok=n, B=B, tok0=32, hw=hw, x_st=D, x_sb=0)
    fr = (torch.arange(n, device=device) + 32) // hw
    hr = F.layer_norm(x.expand(n, B, D), (D,), eps=1e-6) * (1 + sc[:, fr].transpose(0, 1)) + sh[:, fr].transpose(0, 1)
    ok, eq = bf16_ulp_close(h, hr)
    assert ok, eq


def test_final_ln_mod(device):
    n, B, D, T, hw = 40, 2, 1024, 2, 20
    g = torch.Generator().manual_seed(2)
    x = torch.randn(n, B, D, generator=g).to(device, torch.bfloat16)
    y = torch.randn(n, B, D, generator=g).to(device, torch.bfloat16)
    gm = (torch.randn(B, T, 3 * D, generator=g)).to(device, torch.bfloat16)
    f = torch.randn(B, T, 2 * D, generator=g).to(device)
    sh, sc = f.chunk(2, -1)
    out = N.final_ln_mod(x, sh, sc, n_tok=n, B=B, tok0=0, hw=hw, y=y, gate=gm[..., 2 * D:])
    fr = torch.arange(n, device=device) // hw
    xr = x + gm[..., 2 * D:][:, fr].transpose(0, 1) * y
    ref = F.layer_norm(xr.float(), (D,), eps=1e-6) * (1 + sc[:, fr].transpose(0, 1)) + sh[:, fr].transpose(0, 1)
    assert ((out - ref).abs().max() / ref.abs().max()).item() < 1e-5


def test_head_rmsnorm_rope(device):
    n, B, H = 50, 2, 4
    D = H * 128
    g = torch.Generator().manual_seed(3)
    buf = torch.randn(n * B, 3 * D, generator=g).to(device, torch.bfloat16)
    w = (1 + 0.1 * torch.randn(128, generator=g)).to(device, torch.bfloat16)
    fr = torch.rand(n, 64, generator=g).to(device) * 50
    cos, sin = torch.cos(fr), torch.sin(fr)
    ref_in = buf.clone()
    N.head_rmsnorm_rope(buf, n_rows=n * B, B=B, H=H, head_off=D, weight=w, cos=cos, sin=sin)
    k = ref_in[:, D:2 * D].view(n * B, H, 128).float()
    kn = ((k * torch.rsqrt(k.pow(2).mean(-1, keepdim=True) + 1e-6)) * w.float()).to(torch.bfloat16).float()
    f2 = torch.cat([fr, fr], -1).repeat_interleave(B, 0)[:, None, :]
    rot = torch.cat([-kn[..., 64:], kn[..., :64]], -1)
    ref = (kn * torch.cos(f2) + rot * torch.sin(f2)).to(torch.bfloat16)
    ok, eq = bf16_ulp_close(buf[:, D:2 * D].view(n * B, H, 128), ref)
    assert ok, eq
    assert torch.equal(buf[:, :D], ref_in[:, :D]) and torch.equal(buf[:, 2 * D:], ref_in[:, 2 * D:])


def _gelu_exact_bf16(x):
    """float64 x * Phi(x) with Phi = erfc(-x / sqrt 2) / 2 (no 1 + erf cancellation), rounded once to bf16."""
    xd = x.double().cpu()
    return (xd * 0.5 * torch.special.erfc(-xd * 0.5 ** 0.5)).to(torch.bfloat16)


def _check_gelu(x, y):
    """cp25_gelu (cp25_common.h gelu_erf) vs the correctly rounded GELU: within one bf16 ulp everywhere, equal on
    >= 99.9 % of inputs. Outputs below the fp32 normal range may flush to zero on the GPU. torch's own GELU
    (x/2 (1 + erf(x / sqrt 2)), what the reference's nn.GELU runs) cancels for x << 0: it is compared only on
    x >= -2, where it is accurate."""
    ref = _gelu_exact_bf16(x).to(y.device)
    keep = ref.float().abs() >= 2.0 ** -126
    ok, eq = bf16_ulp_close(y[keep], ref[keep])
    assert ok, eq
    assert (y[~keep].float().abs() <= 2.0 ** -126).all()
    mild = x >= -2
    ok_t, eq_t = bf16_ulp_close(y[mild], F.gelu(x[mild]))
    assert ok_t, eq_t


def test_gelu(device):
    x = (torch.randn(4096 * 3) * 3).to(device, torch.bfloat16)
    y = x.clone()
    N.gelu_(y)
    _check_gelu(x, y)


def test_gelu_every_bf16_value(device):
    """Exact-erf GELU over every finite bf16 input (65 024 values)."""
    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    x = bits[torch.isfinite(bits.float())].to(device)
    y = x.clone()
    N.gelu_(y)
    _check_gelu(x, y)


def test_patchify_and_cfg_exact(device):
    T, Hp, Wp = 3, 4, 6
    L, hw = T * Hp * Wp, Hp * Wp
    g = torch.Generator().manual_seed(4)
    xs = torch.randn(L, 64, generator=g).to(device)
    gt = torch.randn(L, 64, generator=g).to(device)
    noise = torch.randn(L, 64, generator=g).to(device)
    fm = torch.tensor([1.0, 0.0, 0.0], device=device)
    rows = N.patchify(xs, gt, fm, None, tok0=0, hw=hw)
    m = fm[torch.arange(L, device=device) // hw][:, None]
    xin = (gt * m + xs * (1 - m)).to(torch.bfloat16)  # [L, (p c)]
    ref = torch.zeros(L, 72, dtype=torch.bfloat16, device=device)
    ref[:, :64] = xin.view(L, 4, 16).transpose(1, 2).reshape(L, 64)
    ref[:, 64:68] = m.to(torch.bfloat16)
    assert torch.equal(rows, ref)
    net = torch.randn(L, 2, 64, generator=g).to(device)
    v = N.cfg_velocity(net, noise, gt, fm, 7.0, 0, tok0=0, hw=hw)
    vb = [(noise - gt) * m + net[:, b] * (1 - m) for b in range(2)]
    assert torch.equal(v, vb[0] + 7.0 * (vb[0] - vb[1]))


@pytest.mark.parametrize("karras,steps", [(True, 35), (False, 35), (True, 2)])
def test_unipc_bit_exact(device, karras, steps):
    """The fused step reproduces the reference's fp32 UniPC trajectory bit for bit (oracle/unipc.py)."""
    n = 4096 + 7
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(n, generator=g)
    orc = UniPC(steps, shift=5.0, use_karras=karras)
    sch = FlowUniPCMultistepScheduler(shift=1)
    sch.set_timesteps(steps, device=device, shift=5.0, use_kerras_sigma=karras)
    assert torch.equal(sch.timesteps.cpu(), orc.timesteps)
    assert torch.equal(sch.sigmas, orc.sigmas)
    xg = sch.begin(x0.to(device))
    xc = x0.clone()
    for i, t in enumerate(orc.timesteps):
        v = torch.sin(xc * 1.3 + i) * 0.7 + 0.1 * torch.randn(n, generator=g)  # fake model output
        xc = orc.step(v, t, xc)
        sch.step_(v.to(device), t)
        assert torch.equal(xg.cpu(), xc), f"step {i}: max diff {(xg.cpu() - xc).abs().max().item()}"


def test_unipc_bit_exact_full_latent(device):
    """The metric's whole latent (16 x 31 x 88 x 160 = 6.98 M elements), 35 Karras steps: the fused
    HIP step stays bit-identical to the fp32 oracle trajectory at full size."""
    n = 16 * 31 * 88 * 160
    steps = 35
    g = torch.Generator().manual_seed(9)
    x0 = torch.randn(n, generator=g)
    orc = UniPC(steps, shift=5.0, use_karras=True)
    sch = FlowUniPCMultistepScheduler(shift=1)
    sch.set_timesteps(steps, device=device, shift=5.0, use_kerras_sigma=True)
    xg = sch.begin(x0.to(device))
    xc = x0.clone()
    for i, t in enumerate(orc.timesteps):
        v = torch.sin(xc * 1.3 + i) * 0.7
        xc = orc.step(v, t, xc)
        sch.step_(v.to(device), t)
    assert torch.equal(xg.cpu(), xc)
