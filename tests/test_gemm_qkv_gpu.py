"""cp25_gemm_qkv: the fused q|k|v projection with the k columns' per-head RMSNorm + 3D RoPE in the GEMM epilogue must
equal cp25_gemm_epi followed by cp25_head_rmsnorm_rope on the k columns BIT FOR BIT (Attention.compute_qkv's k_proj +
k_norm + apply_rotary_pos_emb, minimal_v4_dit.py:401-419). Token-major rows (tok = row // B), ragged row tiles,
without RoPE, the DiT's metric shape.
"""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,B,H,K,rope", [
    (500, 2, 2, 128, True),       # ragged last row tile (1000 rows), two heads per k tile
    (777, 1, 4, 256, True),       # B = 1, two k tiles
    (640, 2, 2, 128, False),      # no RoPE
    (109120, 2, 16, 2048, True),  # the metric's QKV launch
])
def test_gemm_qkv_bit_identical(device, n, B, H, K, rope):
    g = torch.Generator(device=device).manual_seed(n + H + K)
    D = H * 128
    M = n * B
    a = torch.randn(M, K, device=device, generator=g).to(torch.bfloat16)
    w = (torch.randn(3 * D, K, device=device, generator=g) * K ** -0.5).to(torch.bfloat16)
    kw = (0.5 + 2.5 * torch.rand(128, device=device, generator=g)).to(torch.bfloat16)
    cos = sin = None
    if rope:
        ang = torch.rand(n, 64, device=device, generator=g) * 50.0
        cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    fused = N.gemm_qkv(a, w, kw, k_col0=D, k_cols=D, B=B, cos=cos, sin=sin)
    assert fused is not None
    ref = N.gemm_epi(a, w)
    N.head_rmsnorm_rope(ref, n_rows=M, B=B, H=H, head_off=D, weight=kw, cos=cos, sin=sin)
    assert torch.isfinite(fused.float()).all()
    assert torch.equal(fused, ref), (fused.float() - ref.float()).abs().max().item()


def test_gemm_qkv_rejects(device):
    a = torch.randn(256, 128, device=device).to(torch.bfloat16)
    w = torch.randn(768, 128, device=device).to(torch.bfloat16)
    kw = torch.ones(128, device=device, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        N.gemm_qkv(a, w, kw, k_col0=128, k_cols=256, B=1)  # not a multiple of the 256-column tile
    a3 = torch.randn(256, 192, device=device).to(torch.bfloat16)
    w3 = torch.randn(768, 192, device=device).to(torch.bfloat16)
    assert N.gemm_qkv(a3, w3, kw, k_col0=256, k_cols=256, B=1) is None  # K / 64 odd: declined
