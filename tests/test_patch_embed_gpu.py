"""The x_embedder on the own GEMM: cp25_patchify_ld writes the patch rows into a zero-padded [n, 128] buffer and the
DiT multiplies them by the weight zero-padded to K = 128 (cp25_gemm_epi) instead of the library's K = 72 GEMM
(PatchEmbed, minimal_v4_dit.py:846-913). The padded rows must equal cp25_patchify's rows with zeros after column
72, and the embedding must match the library linear on the same rows to bf16 rounding (fp32 sums in another order).
"""
import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N
from cosmos_predict2.dit import Geometry, MinimalV1LVGDiT, init_state_dict
from cosmos_predict2.net_config import tiny_dit

pytestmark = pytest.mark.gpu


def test_patchify_ld_rows(device):
    g = torch.Generator(device=device).manual_seed(0)
    n, hw = 1000, 40
    xs = torch.randn(n, 64, device=device, generator=g)
    gt = torch.randn(n, 64, device=device, generator=g)
    mask = (torch.rand(n // hw + 1, device=device, generator=g) > 0.5).float()
    a = N.patchify(xs, gt, mask, None, tok0=0, hw=hw)
    b = N.patchify(xs, gt, mask, None, tok0=0, hw=hw, ld=128)
    assert b.stride(0) == 128 and torch.equal(a, b)
    full = torch.as_strided(b, (n, 128), (128, 1))
    assert torch.equal(full[:, 72:], torch.zeros_like(full[:, 72:]))


def test_embed_patches_own_gemm(device):
    cfg = tiny_dit(num_blocks=1)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict({"net." + k: v for k, v in init_state_dict(cfg, seed=3).items()})
    g = torch.Generator(device=device).manual_seed(1)
    n = 4 * 8 * 8
    xs = torch.randn(n, 64, device=device, generator=g)
    mask = torch.ones(4, device=device)
    rows = N.patchify(xs, None, mask, None, tok0=0, hw=64, ld=128)
    geo = Geometry(T=4, Hp=8, Wp=8, tok0=0, n_tok=n, n_views=1)
    own = net.embed_patches(rows.view(n, 1, 72), geo, rows_k128=True)
    lib = F.linear(rows.contiguous(), net.sd["x_embedder.proj.1.weight"]).view(n, 1, -1)
    assert own.dtype == torch.bfloat16 and own.shape == lib.shape
    diff = (own.float() - lib.float()).abs()
    ulp = lib.float().abs().clamp_min(1e-3) * 2.0 ** -7
    assert (diff <= ulp).all(), diff.max().item()
    # without the flag the 72 columns are copied into a zero-padded operand (never read from the padded storage): the
    # same operand, the same GEMM, the same bits; likewise per batch entry for [n, 2, 72] rows
    assert torch.equal(net.embed_patches(rows.view(n, 1, 72), geo), own)
    rows2 = torch.stack([rows, rows.flip(0)], 1).contiguous()
    two = net.embed_patches(rows2, geo)
    assert two.shape == (n, 2, own.shape[-1])
    assert torch.equal(two[:, :1], own) and torch.equal(two[:, 1:], net.embed_patches(rows.flip(0).view(n, 1, 72), geo))
