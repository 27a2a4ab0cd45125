"""cp25_attn_fwd_prescaled_qnorm: the self-attention normalising its own q (per-head RMSNorm + rotate-half RoPE +
the prescale, applied to the Q fragments as they load) must equal cp25_head_rmsnorm_rope_scaled on q followed by
cp25_attn_fwd_prescaled BIT FOR BIT: same partial-sum order, same roundings (the DiT's default path since round 4,
replacing the separate q pass; Attention.compute_qkv's q_norm + RoPE, minimal_v4_dit.py:401-419).

Covers the DiT's fused [n, B, 3D] layout, ragged query blocks, the three softmax modes (zero shift, fixed shift,
online max), no RoPE (cross-attention-style q), the tail-split launch (its sub-problems index the RoPE tables from
their first query row) and the gated k-slot pair.
"""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

HD = 128
C = HD ** -0.5 * 1.4426950408889634


def _qkv(device, n, B, H, seed, wlo=0.5, whi=3.0, rope=True):
    g = torch.Generator(device=device).manual_seed(seed)
    D = H * HD
    qkv = (torch.randn(n, B, 3 * D, device=device, generator=g) * 3.0).to(torch.bfloat16)
    wq = (wlo + (whi - wlo) * torch.rand(HD, device=device, generator=g)).to(torch.bfloat16)
    wk = (wlo + (whi - wlo) * torch.rand(HD, device=device, generator=g)).to(torch.bfloat16)
    cos = sin = None
    if rope:
        ang = torch.rand(n, 64, device=device, generator=g) * 50.0
        cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    flat = qkv.view(n * B, 3 * D)
    N.head_rmsnorm_rope(flat, n_rows=n * B, B=B, H=H, head_off=D, weight=wk, cos=cos, sin=sin)  # k as the DiT does
    return qkv, wq, cos, sin


def _views(qkv, n, B, H):
    D = H * HD
    q, k, v = (qkv[:, :, i * D:(i + 1) * D].view(n, B, H, HD).transpose(0, 1) for i in range(3))
    return q, k, v


def _both(qkv, wq, cos, sin, n, B, H, **kw):
    D = H * HD
    q, k, v = _views(qkv, n, B, H)
    fused = N.attn_fwd(q, k, v, prescaled=True, q_norm=dict(weight=wq, cos=cos, sin=sin, out_scale=C), **kw)
    q2 = qkv.clone()
    N.head_rmsnorm_rope(q2.view(n * B, 3 * D), n_rows=n * B, B=B, H=H, head_off=0, weight=wq, cos=cos, sin=sin,
                        out_scale=C)
    qr, _, _ = _views(q2, n, B, H)
    ref = N.attn_fwd(qr, k, v, prescaled=True, **kw)
    return fused, ref


@pytest.mark.parametrize("n,B,H,bounds,rope", [
    (1000, 2, 2, "zero", True),    # ragged last query block, zero shift
    (777, 1, 3, "fixed", True),    # fixed per-row shift
    (1300, 2, 2, "online", True),  # no bounds: online max
    (640, 2, 2, "zero", False),    # no RoPE
])
def test_qnorm_in_kernel_bit_identical(device, n, B, H, bounds, rope):
    qkv, wq, cos, sin = _qkv(device, n, B, H, seed=n + H, rope=rope)
    qb = HD ** 0.5 * float(wq.float().abs().max()) * C * 1.001
    kb = HD ** 0.5 * 3.0 * 1.001
    if bounds == "zero":  # shrink the q weights until the weight bound allows the zero shift
        wq = (wq.float() * (95.0 / (qb * kb))).to(torch.bfloat16)
        nb = (HD ** 0.5 * float(wq.float().abs().max()) * C * 1.001, kb)
        assert nb[0] * nb[1] <= 96.0
    elif bounds == "fixed":
        nb = (97.0 / kb, kb)  # product 97 picks the fixed shift (per row from its own |q| and the true key bound)
    else:
        nb = None
    fused, ref = _both(qkv, wq, cos, sin, n, B, H, norm_bounds=nb)
    assert torch.isfinite(fused.float()).all()
    assert torch.equal(fused, ref), (fused.float() - ref.float()).abs().max().item()


def test_qnorm_tail_split_rope_rows(device):
    """The unsplit launch of a shape whose last partial round runs as tail splits (B = H = 1 sub-problems of the
    last query blocks): their RoPE rows are token row0 + row, not row."""
    B, H, Lq, Lk = 1, 16, 13640, 32768
    assert N.load_library().cp25_attn_tail_workspace_bytes(B, H, Lq, Lk) > 0  # the plan has a tail here
    g = torch.Generator(device=device).manual_seed(5)
    D = H * HD
    qraw = (torch.randn(Lq, B, D, device=device, generator=g) * 2.0).to(torch.bfloat16)
    kv = torch.randn(Lk, B, 2 * D, device=device, generator=g).to(torch.bfloat16)
    wk = torch.ones(HD, device=device, dtype=torch.bfloat16)
    N.head_rmsnorm_rope(kv.view(Lk * B, 2 * D), n_rows=Lk * B, B=B, H=H, head_off=0, weight=wk)
    wq = (0.5 + torch.rand(HD, device=device, generator=g)).to(torch.bfloat16)
    ang = torch.rand(Lq, 64, device=device, generator=g) * 50.0
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    k = kv[:, :, :D].view(Lk, B, H, HD).transpose(0, 1)
    v = kv[:, :, D:].view(Lk, B, H, HD).transpose(0, 1)
    q = qraw.view(Lq, B, H, HD).transpose(0, 1)
    fused = N.attn_fwd(q, k, v, prescaled=True, q_norm=dict(weight=wq, cos=cos, sin=sin, out_scale=C))
    q2 = qraw.clone()
    N.head_rmsnorm_rope(q2.view(Lq * B, D), n_rows=Lq * B, B=B, H=H, head_off=0, weight=wq, cos=cos, sin=sin,
                        out_scale=C)
    ref = N.attn_fwd(q2.view(Lq, B, H, HD).transpose(0, 1), k, v, prescaled=True)
    assert torch.equal(fused, ref), (fused.float() - ref.float()).abs().max().item()


def test_qnorm_gated_kslots(device):
    """The gated pair (data-tight key bound in device slots) with the in-kernel q normalisation."""
    n, B, H = 1500, 2, 2
    D = H * HD
    qkv, wq, cos, sin = _qkv(device, n, B, H, seed=11, wlo=2.0, whi=3.0)
    slots = torch.zeros(64, 32, device=device, dtype=torch.float32)
    flat = qkv.view(n * B, 3 * D)
    N.head_rmsnorm_rope(flat, n_rows=n * B, B=B, H=H, head_off=D, weight=torch.ones(HD, device=device,
                        dtype=torch.bfloat16), norm_max=slots)  # k rows normed again (unit weight) + their max
    nb = (HD ** 0.5 * 3.0 * C * 1.001, HD ** 0.5 * 1.001 * 3.0)
    fused, ref = _both(qkv, wq, cos, sin, n, B, H, norm_bounds=nb, k_norm_slots=slots)
    assert torch.equal(fused, ref), (fused.float() - ref.float()).abs().max().item()


def test_qnorm_rejects_bad_arguments(device):
    qkv, wq, cos, sin = _qkv(device, 64, 1, 1, seed=1)
    q, k, v = _views(qkv, 64, 1, 1)
    with pytest.raises(ValueError):
        N.attn_fwd(q, k, v, q_norm=dict(weight=wq, cos=cos, sin=sin))  # not prescaled
    with pytest.raises(ValueError):
        N.attn_fwd(q, k, v, prescaled=True, q_norm=dict(weight=wq, cos=cos, sin=None))
    with pytest.raises(ValueError):
        N.attn_fwd(q, k, v, prescaled=True, q_norm=dict(weight=wq.float(), cos=cos, sin=sin))
