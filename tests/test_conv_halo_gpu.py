"""The 3x3 halo conv (conv3x3_halo_kernel: LDS halo tile per (temporal tap, 16-channel chunk), the 9 spatial taps
read from it) vs fp32 math and vs the per-tap implicit-GEMM kernel (cp25_conv3d_select(1)).

Reference: CausalConv3d (tokenizers/wan2pt1.py:44-62) and the Resample upsample conv (:96-110). The halo
kernel sums the same products in another order (channel chunk outer, tap inner), so it is held to the
single-conv bound vs fp32 (rel-L2 <= 2e-3, one bf16 output rounding) and to <= 2e-3 vs the per-tap kernel.
Shapes cover the three tile widths (Wo % 128, % 64, % 32), a ragged last row-tile, a causal zero frame, the
nearest-2x upsample gather, bias + residual, and Cout = 192 / 384 (several 96-channel tiles).
"""
import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N
from cosmos_predict2.vae import _Conv

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def _both(fn):
    """(the default halo kernel's output, the per-tap kernel's); the 4-wave form of the halo kernel must equal the
    default 8-wave one bit for bit (same taps, same channel-chunk order, same MFMA chains per output)."""
    out = fn()
    prev = N.conv3d_select(1)
    try:
        ref = fn()
        N.conv3d_select(2)
        out4 = fn()
    finally:
        N.conv3d_select(prev)
    assert torch.equal(out4, out)
    return out, ref


@pytest.mark.parametrize("cin,cout,H,W,up", [(96, 96, 9, 128, False), (96, 96, 12, 64, False),
                                             (96, 96, 17, 32, False), (192, 96, 6, 16, True),
                                             (384, 384, 5, 32, False), (96, 192, 8, 96, False)])
def test_conv3x3_halo_2d(device, cin, cout, H, W, up):
    g = torch.Generator().manual_seed(cin * 7 + cout + H + W)
    x = torch.randn(1, cin, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5).to(torch.bfloat16)
    b = (0.1 * torch.randn(cout, generator=g)).to(torch.bfloat16)
    xi = F.interpolate(x.float(), scale_factor=2.0, mode="nearest-exact") if up else x.float()
    ref = F.conv2d(xi, w.float(), b.float(), padding=1)
    conv = _Conv(w, b, device)
    xl = x[0].permute(1, 2, 0).contiguous().to(device)
    out, tap = _both(lambda: conv([xl], 1, H, W, pad=(1, 1, 1, 1), upsample=up))
    e_ref = _rel(out[0].permute(2, 0, 1).cpu(), ref[0])
    e_tap = _rel(out, tap)
    print(f"halo conv {cin}->{cout} {H}x{W} up={up}: rel-L2 vs fp32 {e_ref:.2e}, vs per-tap kernel {e_tap:.2e}")
    assert e_ref <= 2e-3 and e_tap <= 2e-3, (e_ref, e_tap)


def test_conv3x3x3_halo_causal_residual(device):
    """3x3x3 over [zero frame | cache frame | 3 new frames] with bias and a residual, 4 output frames."""
    g = torch.Generator().manual_seed(11)
    C, H, W = 96, 10, 64
    cache = torch.randn(1, C, 1, H, W, generator=g).to(torch.bfloat16)
    x = torch.randn(1, C, 3, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, 3, generator=g) / (27 * C) ** 0.5).to(torch.bfloat16)
    b = (0.1 * torch.randn(C, generator=g)).to(torch.bfloat16)
    res = torch.randn(1, C, 3, H, W, generator=g).to(torch.bfloat16)
    clip = torch.cat([torch.zeros(1, C, 1, H, W), cache.float(), x.float()], 2)
    ref = F.conv3d(F.pad(clip, (1, 1, 1, 1, 0, 0)), w.float(), b.float()).to(torch.bfloat16)
    ref = (ref.float() + res.float()).to(torch.bfloat16)
    conv = _Conv(w, b, device)
    cl = cache[0].permute(1, 2, 3, 0).contiguous().to(device)
    xl = x[0].permute(1, 2, 3, 0).contiguous().to(device)
    rl = res[0].permute(1, 2, 3, 0).contiguous().to(device)
    out, tap = _both(lambda: conv([None, cl[0], xl[0], xl[1], xl[2]], 3, H, W, pad=(1, 1, 1, 1), residual=rl))
    e_ref = _rel(out.permute(3, 0, 1, 2).cpu(), ref[0])
    e_tap = _rel(out, tap)
    print(f"halo conv3d causal + residual: rel-L2 vs fp32 {e_ref:.2e}, vs per-tap kernel {e_tap:.2e}")
    assert e_ref <= 2e-3 and e_tap <= 2e-3, (e_ref, e_tap)
