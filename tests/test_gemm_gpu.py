"""cp25_gemm_epi (the DiT block projections as hand-written MFMA GEMMs) vs fp32 math.

Reference: nn.Linear (no bias) of networks/minimal_v4_dit.py Attention (:354-363, :401-404, :432) and
GPT2FeedForward (:227-254: layer1 -> exact GELU -> layer2), bf16 operands with fp32 accumulation and one
bf16 rounding. Bounds: rel-L2 <= 4e-3 vs fp32 math (one bf16 output rounding ~2e-3); the GELU epilogue is
bit-exact vs cp25_gelu applied to the kernel's own plain product; the gated-residual epilogue (cp25_gemm_res)
bit-exact vs x + gate * y with the reference's two bf16 roundings on the kernel's own product; ragged M (rows past
the last tile). Every row is computed the same way whatever M is (the property that makes a context-parallel
shard's rows equal the full run's): a row prefix of the problem gives the same rows bit for bit.
"""
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
    m2 = max(1, M // 3 + 7)
    assert torch.equal(N.gemm_epi(a[:m2].contiguous(), w), out[:m2])  # row results independent of M


@pytest.mark.parametrize("K", [64, 2048])
def test_gelu_epilogue_every_bf16_value(device, K):
    """The GELU epilogue over every finite bf16 product (65 024 values; the epilogue's table range and the gelu_erf
    fallback outside it) bit-identical to cp25_gelu: A's column 0 holds the values, W's column 0 is 1, so every
    product is the value itself (one exact bf16 rounding) in each of the 256 output columns. K = 2048 runs the
    persistent kernel (K / 64 even), K = 64 the one-tile-per-workgroup kernel."""
    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    x = bits[torch.isfinite(bits.float())].to(device)
    a = torch.zeros(x.numel(), K, dtype=torch.bfloat16, device=device)
    a[:, 0] = x
    w = torch.zeros(256, K, dtype=torch.bfloat16, device=device)
    w[:, 0] = 1.0
    assert torch.equal(N.gemm_epi(a, w)[:, 0], x)
    g = N.gemm_epi(a, w, epilogue=N.EPI_GELU)
    ref = x.clone()
    N.gelu_(ref)
    assert torch.equal(g, ref[:, None].expand(-1, 256))


def test_gemm_strided_output_and_bad_shapes(device):
    a = torch.randn(300, 128, device=device).to(torch.bfloat16)
    w = torch.randn(512, 128, device=device).to(torch.bfloat16)
    big = torch.zeros(300, 1024, device=device, dtype=torch.bfloat16)
    N.gemm_epi(a, w, out=big[:, 256:768])
    assert torch.equal(big[:, 256:768], N.gemm_epi(a, w))
    assert (big[:, :256] == 0).all() and (big[:, 768:] == 0).all()
    with pytest.raises(ValueError):
        N.gemm_epi(a, torch.randn(300, 128, device=device).to(torch.bfloat16))  # N not a multiple of 256


def _rbf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("M,Nn,K,B,hw,tok0,xsb0", [(1000, 256, 64, 2, 40, 0, False), (2048, 2048, 2048, 2, 64, 96, False),
                                                  (515, 512, 8192, 1, 16, 5, False), (777, 2048, 2048, 2, 300, 13, True),
                                                  (4352, 2048, 8192, 2, 3520, 0, False), (300, 256, 192, 1, 7000, 0, False)])
def test_gemm_residual_epilogue(device, M, Nn, K, B, hw, tok0, xsb0):
    """cp25_gemm_res: x' = x + gate * (a w^T) per token-major row (tok, b) = (r / B, r % B), gate by the row's frame
    (tok0 + tok) / hw, x broadcast over the batch when x_sb = 0 (the CFG pair's shared block-0 rows); ragged M, odd
    K / 64 (the two-phase kernel), shard offsets inside a frame."""
    g = torch.Generator(device=device).manual_seed(M + K + B)
    Mp = (M + B - 1) // B * B
    a = torch.randn(Mp, K, device=device, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=device, generator=g) * K ** -0.5).to(torch.bfloat16)
    n_tok = Mp // B
    T = (tok0 + n_tok - 1) // hw + 1
    gate = (torch.randn(B, T, 3 * Nn, device=device, generator=g)).to(torch.bfloat16)[..., 2 * Nn:]  # a mods view
    Bx = 1 if xsb0 else B
    x = torch.randn(n_tok, Bx, Nn, device=device, generator=g).to(torch.bfloat16)
    out = N.gemm_res(a, w, x, x.stride(0), 0 if xsb0 else x.stride(1), gate, B=B, tok0=tok0, hw=hw)
    y = N.gemm_epi(a, w).float().view(n_tok, B, Nn)
    fr = (tok0 + torch.arange(n_tok, device=device)) // hw
    gr = gate.float()[:, fr].transpose(0, 1)  # [n_tok, B, N]
    ref = _rbf(x.float().expand(n_tok, B, Nn) + _rbf(gr * y))
    assert torch.equal(out.view(n_tok, B, Nn).float(), ref)
    with pytest.raises(ValueError):
        N.gemm_res(a, w, x, x.stride(0), 0, gate[:, :1], B=B, tok0=tok0 + hw * T, hw=hw)  # frames past the gate


@pytest.mark.parametrize("M,Nn,K", [(1000, 256, 512), (2048, 2048, 2048), (515, 6144, 2048), (4352, 2048, 8192),
                                    (777, 8192, 2048)])
def test_gemm_fp8_matches_dequantised(device, M, Nn, K):
    """cp25_gemm_fp8 (config 5's fp8 option; the reference has no fp8 path): bf16((q w8^T) * s_row * s_col) on
    v_mfma_scale_f32_16x16x128_f8f6f4 against the same product in fp32 on the dequantised operands (one bf16 output
    rounding, rel-L2 <= 4e-3) and against torch._scaled_mm (hipBLASLt) on the same operands; rows independent of M;
    the residual epilogue bit-exact vs x + gate * y on the kernel's own product."""
    g = torch.Generator(device=device).manual_seed(M + Nn + K)
    x = torch.randn(M, K, device=device, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=device, generator=g) * K ** -0.5).to(torch.bfloat16)
    q, s = N.quant_fp8_rows(x)
    fmax = torch.finfo(torch.float8_e4m3fn).max
    ws = (w.float().abs().amax(1, keepdim=True) / fmax).clamp_min(1e-30)
    w8 = (w.float() / ws).clamp(-fmax, fmax).to(torch.float8_e4m3fn)
    wsr = ws.t().contiguous()
    out = N.gemm_fp8(q, s, w8, wsr)
    ref = (q.float() * s) @ (w8.float() * ws).t()
    lib = torch._scaled_mm(q, w8.t(), scale_a=s, scale_b=wsr, out_dtype=torch.bfloat16)
    e, el, d = _rel(out, ref), _rel(lib, ref), _rel(out, lib)
    print(f"gemm fp8 M={M} N={Nn} K={K}: vs dequantised fp32 {e:.2e} (torch._scaled_mm {el:.2e}), own vs lib {d:.2e}")
    assert torch.isfinite(out.float()).all()
    assert e <= 4e-3, e
    assert d <= 6e-3, d
    m2 = M // 3 + 5
    assert torch.equal(N.gemm_fp8(q[:m2].contiguous(), s[:m2].contiguous(), w8, wsr), out[:m2])
    B, hw = 1, 64
    gate = torch.randn(1, (M + hw - 1) // hw, Nn, device=device, generator=g).to(torch.bfloat16)
    xr = torch.randn(M, 1, Nn, device=device, generator=g).to(torch.bfloat16)
    o2 = N.gemm_fp8(q, s, w8, wsr, res=(xr, xr.stride(0), xr.stride(1), gate, B, 0, hw))
    fr = torch.arange(M, device=device) // hw
    exp = _rbf(xr[:, 0].float() + _rbf(gate[0, fr].float() * out.float()))
    assert torch.equal(o2.float(), exp)


def _tail_plan(M, Nn, cus):
    """The persistent kernel's tail plan (gemm.hip `plan`): whole tiles, or the last round as half / quarter slices."""
    tiles = (M + 255) // 256 * (Nn // 256)
    P = min(4 * tiles, cus)
    R = tiles % P
    return "full" if R == 0 else ("quarter" if 4 * R <= P else ("half" if 2 * R <= P else "whole"))


def test_gemm_rows_independent_of_tail_plan(device):
    """Round 6's tail row slices (gemm.hip `plan`): a row computed in a whole tile, a half slice or a quarter slice is
    the same MFMA chain, so every row is bit-identical whichever plan its launch's M gives it. Row prefixes of one
    problem at M values that put the launch in each plan (full rounds only, quarter / half slices for the last round,
    whole tiles in a partial last round), on the persistent K = 2048 kernel, plain / GELU / gated-residual epilogues."""
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    cus = cus & ~7 if cus >= 8 else cus
    Nn, K = 2048, 2048
    pick = {}
    for mt in range(cus // 8, 8 * cus // 8 + 1):  # at least one full round of tiles
        M = mt * 256 - 37  # ragged last tile row
        pick.setdefault(_tail_plan(M, Nn, cus), M)
    assert set(pick) == {"full", "quarter", "half", "whole"}, pick
    Mb = max(pick.values())
    g = torch.Generator(device=device).manual_seed(11)
    a = torch.randn(Mb, K, device=device, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=device, generator=g) * K ** -0.5).to(torch.bfloat16)
    hw = 4096
    gate = torch.randn(1, (Mb + hw - 1) // hw, Nn, device=device, generator=g).to(torch.bfloat16)
    x = torch.randn(Mb, 1, Nn, device=device, generator=g).to(torch.bfloat16)
    full = {e: N.gemm_epi(a, w, epilogue=e) for e in (N.EPI_NONE, N.EPI_GELU)}
    full_res = N.gemm_res(a, w, x, x.stride(0), x.stride(1), gate, B=1, tok0=0, hw=hw)
    for plan, M in sorted(pick.items(), key=lambda kv: kv[1]):
        for e in (N.EPI_NONE, N.EPI_GELU):
            assert torch.equal(N.gemm_epi(a[:M], w, epilogue=e), full[e][:M]), (plan, M, e)
        r = N.gemm_res(a[:M], w, x[:M], x.stride(0), x.stride(1), gate, B=1, tok0=0, hw=hw)
        assert torch.equal(r, full_res[:M]), (plan, M, "res")
    print(f"tail plans on {cus} CUs: {pick}")
