"""gemm_nt_4w (4 waves of 128 x 128, one wave per SIMD; cp25_gemm_select(1)) against gemm_nt_8ph (the round-4 kernel,
8 waves of 128 x 64): every output is the same MFMA chain in the same K order, so the two must agree bit for bit, for
every epilogue (plain, exact GELU, gated residual, head RMSNorm, the fused QKV with k norm + RoPE), ragged row tiles,
several tiles per workgroup (the pipelined tile seam) and B = 1 / 2 residual row groupings. The 8ph kernel itself is
checked against the bf16 linear in tests/test_gemm_gpu.py (minimal_v4_dit.py:227-254, 400-432)."""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _both(fn):
    prev = N.gemm_select(0)
    try:
        ref = fn()
        N.gemm_select(1)
        got = fn()
    finally:
        N.gemm_select(prev)
    return ref, got


def _ops(M, Nn, K, g, dev):
    a = torch.randn(M, K, generator=g, device=dev).to(BF16)
    w = (torch.randn(Nn, K, generator=g, device=dev) * K ** -0.5).to(BF16)
    return a, w


@pytest.mark.parametrize("M,Nn,K", [(4096, 512, 256), (1000, 768, 128), (300, 256, 512), (70000, 2048, 2048),
                                    (13640, 6144, 2048)])
@pytest.mark.parametrize("epi", ["none", "gelu"])
def test_gemm_4w_epi_bit_identical(device, M, Nn, K, epi):
    g = torch.Generator(device=device).manual_seed(M + Nn)
    a, w = _ops(M, Nn, K, g, device)
    e = N.EPI_GELU if epi == "gelu" else N.EPI_NONE
    ref, got = _both(lambda: N.gemm_epi(a, w, epilogue=e))
    assert torch.equal(ref, got), (ref.float() - got.float()).abs().max().item()


@pytest.mark.parametrize("M,Nn,K,B,hw", [(4096, 512, 256, 2, 64), (998, 256, 128, 2, 8), (2560, 2048, 2048, 1, 40),
                                         (13640, 2048, 8192, 1, 3520)])
def test_gemm_4w_res_bit_identical(device, M, Nn, K, B, hw):
    g = torch.Generator(device=device).manual_seed(7 + M)
    a, w = _ops(M, Nn, K, g, device)
    n = M // B
    T = (n + hw - 1) // hw + 1
    x = torch.randn(n, B, Nn, generator=g, device=device).to(BF16)
    gate = torch.randn(B, T, Nn, generator=g, device=device).to(BF16)
    ref, got = _both(lambda: N.gemm_res(a, w, x, B * Nn, Nn, gate, B=B, tok0=0, hw=hw))
    assert torch.equal(ref, got), (ref.float() - got.float()).abs().max().item()


@pytest.mark.parametrize("M", [4096, 1000])
def test_gemm_4w_hnorm_qkv_bit_identical(device, M):
    g = torch.Generator(device=device).manual_seed(11 + M)
    a, w = _ops(M, 768, 256, g, device)
    nw = (0.5 + torch.rand(128, generator=g, device=device)).to(BF16)
    ref, got = _both(lambda: N.gemm_hnorm(a, w, nw, out_scale=0.3))
    assert torch.equal(ref, got)
    B = 2
    ang = torch.rand(M // B, 64, generator=g, device=device) * 20
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    ref, got = _both(lambda: N.gemm_qkv(a, w, nw, k_col0=256, k_cols=256, B=B, cos=cos, sin=sin))
    assert torch.equal(ref, got)
    ref, got = _both(lambda: N.gemm_qkv(a, w, nw, k_col0=256, k_cols=256, B=B))
    assert torch.equal(ref, got)
