"""Persistent short-KV attention (cp25_attn_fwd_prescaled at Lk <= 1024: the DiT's text cross-attention,
minimal_v4_dit.py:1216-1226, attention.py:90-181): one workgroup per CU runs a run of query blocks of one (b, h)
as a single key-tile stream (opt-in, CP25_XATTN_KERNEL=persist, read per launch). Same per-block arithmetic as
the one-workgroup-per-block 32x32x16 kernel (attn_fwd_d128, CP25_ATTN_MFMA=32; the default per-block kernel is
the 16x16x32 attn_fwd_m16, tests/test_attn_m16_gpu.py), so the two are compared bit for bit, and both against
fp32 math.
Covers ragged key tiles, one-tile blocks (Lk <= 64), ragged query blocks, chunks of one block, and strided
token-major views as the DiT passes them."""
import os

import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

C = 128 ** -0.5 * 1.4426950408889634


def _normed(shape, g, device):
    t = torch.randn(shape, generator=g)
    return (t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + 1e-6)).to(device, torch.bfloat16)


def _select(blocks):
    os.environ["CP25_XATTN_KERNEL" if not blocks else "CP25_ATTN_MFMA"] = "persist" if not blocks else "32"


def _unselect():
    os.environ.pop("CP25_XATTN_KERNEL", None)
    os.environ.pop("CP25_ATTN_MFMA", None)


def _run(q, k, v, nb, blocks):
    _select(blocks)
    try:
        return N.attn_fwd(q, k, v, norm_bounds=nb, prescaled=True, n_split=1)
    finally:
        _unselect()


@pytest.mark.parametrize("B,H,Lq,Lk", [(2, 16, 20000, 512), (1, 2, 777, 300), (1, 3, 5000, 64), (2, 4, 3333, 1000),
                                       (1, 1, 100, 512), (2, 16, 109120, 512)])
def test_xattn_persistent_bit_exact_and_fp32(device, B, H, Lq, Lk):
    g = torch.Generator().manual_seed(Lq + Lk)
    q = _normed((B, Lq, H, 128), g, device)
    k = _normed((B, Lk, H, 128), g, device)
    v = torch.randn((B, Lk, H, 128), generator=g).to(device, torch.bfloat16)
    qs = (q.float() * C).to(torch.bfloat16)
    nb = (128 ** 0.5 * 1.02 * C, 128 ** 0.5 * 1.02)
    op = _run(qs, k, v, nb, blocks=False)
    ob = _run(qs, k, v, nb, blocks=True)
    assert torch.equal(op, ob)
    rows = slice(0, min(Lq, 4096))  # fp32 reference on a query slice (the full 109 120 x 512 fits, but is slow)
    s = torch.einsum("bqhd,bkhd->bhqk", qs[:, rows].float(), k.float())
    ref = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s * 0.6931471805599453, -1), v.float())
    e = ((op[:, rows].float() - ref).norm() / ref.norm()).item()
    assert e <= 4e-3, e


def test_xattn_persistent_strided_views(device):
    """q / out as [n, B, H, 128] token-major views of [n, B, D] buffers, k / v [B, 512, H, 128] (the DiT's
    cross-attention call, _cross_attention)."""
    B, H, n, Lk = 2, 16, 9000, 512
    g = torch.Generator().manual_seed(5)
    q = (_normed((n, B, H, 128), g, device).float() * C).to(torch.bfloat16)
    k = _normed((B, Lk, H, 128), g, device)
    v = torch.randn((B, Lk, H, 128), generator=g).to(device, torch.bfloat16)
    nb = (128 ** 0.5 * 1.02 * C, 128 ** 0.5 * 1.02)
    outs = []
    for blocks in (False, True):
        o = torch.full((n, B, H * 128), float("nan"), device=device, dtype=torch.bfloat16)
        _select(blocks)
        try:
            N.attn_fwd(q.transpose(0, 1), k, v, out=o.view(n, B, H, 128).transpose(0, 1), norm_bounds=nb,
                       prescaled=True)
        finally:
            _unselect()
        outs.append(o)
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])
