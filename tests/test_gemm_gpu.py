"""cp25_gemm_epi (the DiT block projections as hand-written MFMA GEMMs) vs fp32 math.

Reference: nn.Linear (no bias) of networks/minimal_v4_dit.py Attention (:354-363, :401-404, :432) and
GPT2FeedForward (:227-254: layer1 -> exact GELU -> layer2), bf16 operands with fp32 accumulation and one
bf16 rounding. Bounds: rel-L2 <= 4e-3 vs fp32 math (one bf16 output rounding ~2e-3); the GELU epilogue is
bit-exact vs cp25_gelu applied to the kernel's own plain product; ragged M (rows past the last tile). The
8-phase schedule (default; even K/64) and the two-phase loop (odd K/64, or CP25_GEMM_KERNEL=2ph) accumulate in
the same order and must agree bit for bit.
"""
import os

import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("M,Nn,K", [(1000, 256, 64), (700, 256, 192), (257, 512, 2048), (256, 256, 128), (3000, 2048, 2048), (515, 6144, 2048),
                                    (1024, 2048, 8192), (4352, 8192, 2048)])
def test_gemm_matches_fp32(device, M, Nn, K):
    g = torch.Generator(device=device).manual_seed(M + Nn + K)
    a = torch.randn(M, K, device=device, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=device, generator=g) * K ** -0.5).to(torch.bfloat16)
    out = N.gemm_epi(a, w)
    ref = a.float() @ w.float().t()
    e = _rel(out, ref)
    e_lib = _rel(F.linear(a, w), ref)
    print(f"gemm M={M} N={Nn} K={K}: rel-L2 vs fp32 {e:.2e} (hipBLASLt {e_lib:.2e})")
    assert torch.isfinite(out.float()).all()
    assert e <= 4e-3, e
    g_out = N.gemm_epi(a, w, epilogue=N.EPI_GELU)
    plain = out.clone()
    N.gelu_(plain)
    assert torch.equal(g_out, plain)
    if (K // 64) % 2 == 0:
        os.environ["CP25_GEMM_KERNEL"] = "2ph"
        try:
            out2 = N.gemm_epi(a, w)
        finally:
            os.environ.pop("CP25_GEMM_KERNEL")
        assert torch.equal(out, out2)


def test_gemm_strided_output_and_bad_shapes(device):
    a = torch.randn(300, 128, device=device).to(torch.bfloat16)
    w = torch.randn(512, 128, device=device).to(torch.bfloat16)
    big = torch.zeros(300, 1024, device=device, dtype=torch.bfloat16)
    N.gemm_epi(a, w, out=big[:, 256:768])
    assert torch.equal(big[:, 256:768], N.gemm_epi(a, w))
    assert (big[:, :256] == 0).all() and (big[:, 768:] == 0).all()
    with pytest.raises(ValueError):
        N.gemm_epi(a, torch.randn(300, 128, device=device).to(torch.bfloat16))  # N not a multiple of 256
