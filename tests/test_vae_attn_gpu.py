"""cp25_vae_attn (the VAE AttentionBlock's single-head, d = 384 flash kernel) vs fp32 math.

Reference: AttentionBlock.forward (tokenizers/wan2pt1.py:225-261): F.scaled_dot_product_attention on bf16
q / k / v [b*t, 1, h*w, 384] (flash / efficient backends: fp32 scores and sums, bf16 P). Bound rel-L2 <= 4e-3
vs fp32 softmax(q k^T / sqrt(384)) v of the same bf16 inputs (bf16 P + one output rounding; measured printed).
Covers strided column slices of a [T, L, 3C] to_qkv buffer (the product's call), T > 1, ragged Lq / Lk (not a
multiple of the 128-query block or the 32-key tile), Lk != Lq (the banded decode's gathered keys), and a
row whose scores span a wide range: a key far above the first key tile's maximum overflows the one-pass shift,
so its query blocks take the exact-max redo launch.
"""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

C = 384


def _ref(q, k, v):
    s = torch.einsum("tqd,tkd->tqk", q.float(), k.float()) * C ** -0.5
    return torch.einsum("tqk,tkd->tqd", torch.softmax(s, -1), v.float())


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("T,L", [(1, 1280), (2, 1000), (1, 333)])
def test_vae_attn_qkv_slices(device, T, L):
    g = torch.Generator(device=device).manual_seed(T * 7 + L)
    qkv = torch.randn(T, L, 3 * C, device=device, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]
    out = N.vae_attn(q, k, v)
    err = _rel(out, _ref(q, k, v))
    print(f"vae_attn T={T} L={L}: rel-L2 vs fp32 {err:.2e}")
    assert torch.isfinite(out.float()).all()
    assert err <= 4e-3, err


def test_vae_attn_gathered_keys_and_wide_scores(device):
    g = torch.Generator(device=device).manual_seed(3)
    q = torch.randn(1, 512, C, device=device, generator=g).to(torch.bfloat16)
    k = torch.randn(1, 1536, C, device=device, generator=g)
    k[0, 700] *= 6.0  # one key far above the rest: scores of up to ~100 in log2 units
    k = k.to(torch.bfloat16)
    v = torch.randn(1, 1536, C, device=device, generator=g).to(torch.bfloat16)
    out = N.vae_attn(q, k, v)
    err = _rel(out, _ref(q, k, v))
    print(f"vae_attn Lq=512 Lk=1536 (spiked key): rel-L2 vs fp32 {err:.2e}")
    assert torch.isfinite(out.float()).all()
    assert err <= 4e-3, err
    with pytest.raises(ValueError):
        N.vae_attn(q[:, :, :128], k[:, :, :128], v[:, :, :128])  # head dim 128: not this kernel
