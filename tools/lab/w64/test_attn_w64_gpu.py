"""Lab test (round 6): attn_fwd_w64 (one wave per SIMD, 64 query rows per wave; a lab build, not the
product) against attn_fwd_m16 on the same inputs: bit-identical, because both run the same v_mfma_f32_16x16x32_bf16 chains in
the same order on the same operands (attn_w64.hip header). Reference op: networks/attention.py:90-181.

Covers the three softmax-shift modes (zero / fixed / online), ragged query blocks and key tiles, key-range splits
(including one-tile splits), the tail split of a partial last round (its own kernel symbol), the in-kernel q
RMSNorm + RoPE, the DiT's token-major strided views, trained-size norm weights and the metric launch itself.
Run it in its own process on the lab library:
  tools/lab/w64/build_lab.sh lab "" && python -m pytest tools/lab/w64/test_attn_w64_gpu.py -v
"""
import os
import sys

import pytest
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "..", "..", "..", "cosmos-predict2.5_amd"))
from cosmos_predict2 import _native as N  # noqa: E402

_LAB = os.path.join(_HERE, "libcp25_lab.so")
N._LIB_PATH = _LAB
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.exists(_LAB), reason="lab library not built")]

LOG2E = 1.4426950408889634
C = 128 ** -0.5 * LOG2E


def _rms_rows(t, w):
    tf = t.float()
    return (tf * torch.rsqrt(tf.pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16)


def _inputs(device, B, H, Lq, Lk, seed, wlo=0.5, whi=1.5):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w = wlo + (whi - wlo) * torch.rand(128, generator=g)
    q = (_rms_rows(torch.randn(B, Lq, H, 128, generator=g), w).float() * C).to(torch.bfloat16).to(device)
    k = _rms_rows(torch.randn(B, Lk, H, 128, generator=g), w).to(device)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    return q, k, v, w


def _both(fn):
    """fn() under attn_fwd_m16, then under attn_fwd_w64 in every mode (the library's form restored afterwards)."""
    prev = N.attn_self_select(0)
    try:
        a = fn()
        torch.cuda.synchronize()
        N.attn_self_select(2)
        b = fn()
        torch.cuda.synchronize()
    finally:
        N.attn_self_select(prev)
    return a, b


def _modes(q, k):
    qb = q.float().norm(dim=-1).max().item() * 1.01
    kn = k.float().norm(dim=-1).max().item() * 1.01
    return {"zero": (qb, kn), "fixed": (97.0 / kn, kn), "online": None}


SHAPES = [(1, 2, 513, 4100, 1), (2, 2, 1000, 5000, 1), (1, 2, 777, 6000, 3), (1, 1, 300, 4097, 65),
          (2, 3, 256, 4160, 2), (1, 1, 33, 8192, 1), (1, 2, 4800, 4800, 7)]


@pytest.mark.parametrize("B,H,Lq,Lk,n_split", SHAPES)
@pytest.mark.parametrize("mode", ["zero", "fixed", "online"])
def test_w64_bit_identical_to_m16(device, B, H, Lq, Lk, n_split, mode):
    q, k, v, _ = _inputs(device, B, H, Lq, Lk, 11 + Lq + Lk + n_split)
    nb = _modes(q, k)[mode]
    a, b = _both(lambda: N.attn_fwd(q, k, v, prescaled=True, n_split=n_split, norm_bounds=nb))
    name = N.attn_kernel_name(Lk, norm_bounds=nb, prescaled=True)  # the library's default form
    want = {"zero": "attn_fwd_w64<self, prescaled, zero shift>", "fixed": "attn_fwd_w64<self, prescaled, fixed shift>",
            "online": "attn_fwd_m16<self, prescaled, online max>"}[mode]
    assert name == want, name
    assert torch.isfinite(b.float()).all()
    assert torch.equal(a, b), (B, H, Lq, Lk, n_split, mode, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize("mode", ["zero", "online"])
def test_w64_tail_split_bit_identical(device, mode):
    """nwg = 29 query blocks x 9 heads = 261 workgroups on 256 CUs: the last 5 run as the tail split's key-range
    segments (attn_fwd_w64<mode, 1>), merged; the library's plan, unsplit otherwise."""
    B, H, L = 1, 9, 29 * 256 - 100
    q, k, v, _ = _inputs(device, B, H, L, L, 5)
    nb = _modes(q, k)[mode]
    assert N.attn_plan(B, H, L, L, 128) == 1
    a, b = _both(lambda: N.attn_fwd(q, k, v, prescaled=True, norm_bounds=nb))
    assert torch.equal(a, b)


@pytest.mark.parametrize("rope", [True, False])
def test_w64_in_kernel_qnorm_bit_identical(device, rope):
    """cp25_attn_fwd_prescaled_qnorm: q raw, the kernel normalises (RMSNorm + RoPE + prescale) its own fragments."""
    B, H, L = 2, 2, 5000
    g = torch.Generator(device="cpu").manual_seed(9)
    w = (0.5 + torch.rand(128, generator=g)).to(torch.bfloat16)
    q = torch.randn(B, L, H, 128, generator=g).to(device, torch.bfloat16)
    k = _rms_rows(torch.randn(B, L, H, 128, generator=g), w.float()).to(device)
    v = torch.randn(B, L, H, 128, generator=g).to(device, torch.bfloat16)
    ang = torch.rand(L, 64, generator=g) * 50.0
    qn = dict(weight=w.to(device), cos=torch.cos(ang).to(device) if rope else None,
              sin=torch.sin(ang).to(device) if rope else None, out_scale=C)
    wb = 128 ** 0.5 * float(w.float().abs().max()) * 1.02
    for nb in ((wb * C, wb), None):
        a, b = _both(lambda: N.attn_fwd(q, k, v, prescaled=True, norm_bounds=nb, q_norm=qn))
        assert torch.equal(a, b)


def test_w64_token_major_views(device):
    """q / k / v as strided views of the DiT's fused [L, B, 3, H, 128] buffer, the output into a strided view."""
    L, B, H = 4500, 2, 4
    g = torch.Generator(device="cpu").manual_seed(17)
    w = 0.5 + torch.rand(128, generator=g)
    qkv = _rms_rows(torch.randn(L, B, 3, H, 128, generator=g), w)
    qkv[:, :, 0] = (qkv[:, :, 0].float() * C).to(torch.bfloat16)
    qkv = qkv.to(device)
    q, k, v = (qkv[:, :, i].transpose(0, 1) for i in range(3))
    nb = (q.float().norm(dim=-1).max().item() * 1.01, k.float().norm(dim=-1).max().item() * 1.01)

    def run():
        out = torch.empty(L, B, H, 128, device=device, dtype=torch.bfloat16)
        N.attn_fwd(q, k, v, out=out.transpose(0, 1), prescaled=True, norm_bounds=nb)
        return out
    a, b = _both(run)
    assert torch.equal(a, b)


@pytest.mark.parametrize("wrange", [(1.0, 1.0), (0.5, 3.0)])
def test_w64_metric_launch_bit_identical(device, wrange):
    """The metric's launch (B 2, H 16, L = 31 x 44 x 80 = 109 120, the DiT's token-major views, fused q norm):
    unit norm weights (zero shift) and trained-size weights in [0.5, 3] (bound product ~147: online max)."""
    L, B, H = 109120, 2, 16
    g = torch.Generator(device=device).manual_seed(3)
    buf = torch.randn(L, B, 3 * H * 128, device=device, generator=g).to(torch.bfloat16)
    q, k, v = (buf[:, :, i * H * 128:(i + 1) * H * 128].view(L, B, H, 128).transpose(0, 1) for i in range(3))
    lo, hi = wrange
    w = lo + (hi - lo) * torch.rand(128, device=device, generator=torch.Generator(device=device).manual_seed(5))
    k.copy_(_rms_rows(k, w))
    ang = torch.rand(L, 64, device=device, generator=torch.Generator(device=device).manual_seed(6)) * 50.0
    qn = dict(weight=w.to(torch.bfloat16), cos=torch.cos(ang).contiguous(), sin=torch.sin(ang).contiguous(),
              out_scale=C)
    wb = 128 ** 0.5 * float(w.abs().max()) * 1.02
    nb = (wb * C, wb)
    a, b = _both(lambda: N.attn_fwd(q, k, v, prescaled=True, norm_bounds=nb, q_norm=qn))
    assert torch.isfinite(b.float()).all()
    assert torch.equal(a, b), (a.float() - b.float()).abs().max().item()
