"""cp25_gemm_hnorm: the cross-attention q projection with its per-head q RMSNorm (+ the prescale) in the GEMM
epilogue must equal cp25_gemm_epi followed by cp25_head_rmsnorm_rope_scaled BIT FOR BIT (same partial-sum order,
butterfly and roundings; minimal_v4_dit.py:401-404, :411-419, the text cross-attention has no RoPE). Ragged row
tiles, one and several column tiles, the DiT's shape, and the odd-K/64 shapes the kernel declines.
"""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

C = 128 ** -0.5 * 1.4426950408889634


@pytest.mark.parametrize("M,Nn,K,scale", [
    (1000, 256, 128, 1.0),      # ragged last row tile, one column tile, shortest K
    (4096, 2048, 2048, C),      # the DiT's width, prescaled
    (218240, 2048, 2048, C),    # the metric's cross-q launch (109 120 tokens x CFG 2)
])
def test_gemm_hnorm_bit_identical(device, M, Nn, K, scale):
    g = torch.Generator(device=device).manual_seed(M + Nn + K)
    a = torch.randn(M, K, device=device, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=device, generator=g) * K ** -0.5).to(torch.bfloat16)
    nw = (0.5 + 2.5 * torch.rand(128, device=device, generator=g)).to(torch.bfloat16)
    fused = N.gemm_hnorm(a, w, nw, out_scale=scale)
    assert fused is not None
    ref = N.gemm_epi(a, w)
    N.head_rmsnorm_rope(ref, n_rows=M, B=1, H=Nn // 128, head_off=0, weight=nw, out_scale=scale)
    assert torch.isfinite(fused.float()).all()
    assert torch.equal(fused, ref), (fused.float() - ref.float()).abs().max().item()


def test_gemm_hnorm_declines_odd_k_tiles(device):
    a = torch.randn(256, 192, device=device).to(torch.bfloat16)  # K / 64 = 3: the two-phase kernel's shapes
    w = torch.randn(256, 192, device=device).to(torch.bfloat16)
    nw = torch.ones(128, device=device, dtype=torch.bfloat16)
    assert N.gemm_hnorm(a, w, nw) is None
    with pytest.raises(ValueError):
        N.gemm_hnorm(a, w, nw.float())
