"""cp25_gemm_f32 (fp32 MFMA GEMM of the fp32 conditioning layers) against a float64 truth, and the DiT's conditioning
and per-prompt context on the hand-written GEMMs against the library GEMMs they replace.

The reference runs these layers as fp32 F.linear under fp32 autocast (minimal_v4_dit.py:727-788 TimestepEmbedding,
:1136-1154 AdaLN-LoRA, :974-995 final layer); v_mfma_f32_16x16x4_f32 keeps fp32 operands, products and sums, so the
kernel differs from any fp32 GEMM only in summation order. Tolerance: max |err| <= 4e-6 of max |truth| (fp32 sums of
K <= 5120 terms; the measured torch fp32 error is printed beside it). The text-context path (crossattn_proj with its
bias as an extra K column, the cross k/v projections; :1430-1434, :401-404) is compared with the library's bf16
F.linear(+bias): <= 1 bf16 ulp of difference on <= 5 % of the elements (the two GEMMs round the same fp32 sum,
accumulated in different orders)."""
import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu
F64 = torch.float64


def _err(got, truth):
    return ((got.double() - truth).abs().max() / truth.abs().max()).item()


@pytest.mark.parametrize("M,Nn,K,act", [(62, 2048, 2048, 1), (62, 6144, 2048, 0), (62, 21504, 2048, 0),
                                        (20000, 64, 2048, 0), (300, 72, 96, 1), (1, 256, 5120, 0), (129, 4096, 256, 0)])
def test_gemm_f32_plain(device, M, Nn, K, act):
    g = torch.Generator(device=device).manual_seed(M * 7 + Nn)
    a = torch.randn(M, K, generator=g, device=device)
    w = torch.randn(Nn, K, generator=g, device=device) * K ** -0.5
    got = N.gemm_f32(a, w, act=act)
    truth = a.double() @ w.double().t()
    ref = a @ w.t()
    if act:
        truth, ref = F.silu(truth), F.silu(ref)
    e, et = _err(got, truth), _err(ref, truth)
    print(f"gemm_f32 M={M} N={Nn} K={K} act={act}: err {e:.2e} (torch fp32 {et:.2e})")
    assert got.shape == (M, Nn) and e <= 4e-6, (e, et)


def test_gemm_f32_batched_strided_addend(device):
    """The AdaLN-LoRA shape: a1 = column blocks of one [BT, nb3 A] matrix, w [nb3, 3D, A], + the LoRA term [BT, 3D]
    broadcast over the sub-layers."""
    g = torch.Generator(device=device).manual_seed(3)
    BT, nb3, A, D3 = 62, 84, 256, 6144
    a_all = torch.randn(BT, nb3 * A, generator=g, device=device)
    a1 = a_all.view(BT, nb3, A).transpose(0, 1)
    w = torch.randn(nb3, D3, A, generator=g, device=device) * A ** -0.5
    lora = torch.randn(BT, D3, generator=g, device=device)
    got = N.gemm_f32(a1, w, add=lora)
    truth = torch.bmm(a1.double(), w.double().transpose(1, 2)) + lora.double()
    assert got.shape == (nb3, BT, D3) and _err(got, truth) <= 4e-6


def test_gemm_f32_bias_silu_and_column_view_addend(device):
    g = torch.Generator(device=device).manual_seed(4)
    a = torch.randn(500, 512, generator=g, device=device)
    w = torch.randn(192, 512, generator=g, device=device) * 512 ** -0.5
    bias = torch.randn(192, generator=g, device=device)
    got = N.gemm_f32(a, w, add=bias, act=N.ACT_SILU)
    assert _err(got, F.silu(a.double() @ w.double().t() + bias.double())) <= 4e-6
    wide = torch.randn(500, 3 * 192, generator=g, device=device)
    got = N.gemm_f32(a, w, add=wide[:, :192])  # the final layer's lora[:, :2D] addend: a strided column view
    assert _err(got, a.double() @ w.double().t() + wide[:, :192].double()) <= 4e-6


def test_gemm_f32_rows_independent_of_m(device):
    """The final linear of a context-parallel shard: rows of a 13 640 x 2 row shard equal the same rows of the whole
    109 120 x 2 sequence bit for bit (split_k=False, as the DiT calls it)."""
    g = torch.Generator(device=device).manual_seed(6)
    x = torch.randn(218240, 2048, generator=g, device=device)
    w = torch.randn(64, 2048, generator=g, device=device) * 2048 ** -0.5
    full = N.gemm_f32(x, w, split_k=False)
    for r0, n in ((3 * 27280, 27280), (7 * 27280, 27280), (100, 300), (5, 40)):
        assert torch.equal(N.gemm_f32(x[r0:r0 + n], w, split_k=False), full[r0:r0 + n]), (r0, n)


def test_gemm_f32_rejects_unbuilt_shapes(device):
    a = torch.randn(8, 48, device=device)
    w = torch.randn(64, 48, device=device)
    with pytest.raises(ValueError):
        N.gemm_f32(a, w)  # K % 32 != 0
    with pytest.raises(ValueError):
        N.gemm_f32(a.double(), w.double())


def _tiny_net(device, **kw):
    from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict
    from cosmos_predict2.net_config import tiny_dit

    cfg = tiny_dit(num_blocks=2, **kw)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict({"net." + k: v for k, v in init_state_dict(cfg, seed=5, zero_adaln_out=False).items()})
    return net


def test_time_modulation_fp32(device):
    """time_modulation on cp25_gemm_f32 vs the same formula in float64 (TimestepEmbedding + AdaLN-LoRA + final AdaLN)."""
    import math

    net = _tiny_net(device)
    cfg, p = net.cfg, net.sd
    t = torch.tensor([[0.0001, 0.5, 0.7], [0.3, 0.5, 0.9]], device=device) * 1000.0
    mods, shift_f, scale_f = net.time_modulation(t)
    D, B, T = cfg.model_channels, 2, 3
    half = D // 2
    expo = torch.exp(-math.log(10000) * torch.arange(half, dtype=F64, device=device) / half)
    arg = t.flatten().double()[:, None] * expo[None]
    sc = torch.cat([torch.cos(arg), torch.sin(arg)], -1)
    h = F.silu(sc @ p["t_embedder.1.linear_1.weight"].double().t())
    lora = h @ p["t_embedder.1.linear_2.weight"].double().t()
    emb = sc * torch.rsqrt(sc.pow(2).mean(-1, keepdim=True) + 1e-6) * p["t_embedding_norm.weight"].double()
    se = F.silu(emb)
    for i in range(cfg.num_blocks):
        for j, m in enumerate(("self_attn", "cross_attn", "mlp")):
            a1 = se @ p[f"blocks.{i}.adaln_modulation_{m}.1.weight"].double().t()
            ref = a1 @ p[f"blocks.{i}.adaln_modulation_{m}.2.weight"].double().t() + lora
            got = mods[i, j].reshape(B * T, 3 * D)
            assert (got.double() - ref).abs().max().item() <= 2 ** -8 * ref.abs().max().item()  # bf16 rounding
    f2 = (se @ p["final_layer.adaln_modulation.1.weight"].double().t()) @ \
        p["final_layer.adaln_modulation.2.weight"].double().t() + lora[:, : 2 * D]
    got = torch.cat([shift_f, scale_f], -1).reshape(B * T, 2 * D)
    # looser than the GEMM alone: the product's sinusoid is fp32 (cos/sin of arguments up to 900 rad, ~5e-5 absolute
    # apart from the float64 one), measured 6.6e-6
    assert _err(got, f2) <= 3e-5


def test_bias_column_gemm_matches_library_linear(device):
    """prepare_context's crossattn_proj form: bias as one more K column of the hand-written bf16 GEMM + EPI_GELU vs the
    library's F.linear(bias) + GELU. Same fp32 sum, other order: <= 1 bf16 ulp apart, on few elements."""
    g = torch.Generator(device=device).manual_seed(11)
    M, Nn, K = 1024, 1024, 3584
    a = torch.randn(M, K, generator=g, device=device).to(torch.bfloat16)
    w = (torch.randn(Nn, K, generator=g, device=device) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(Nn, generator=g, device=device).to(torch.bfloat16)
    kp = (K + 1 + 63) // 64 * 64
    a2 = torch.zeros(M, kp, dtype=torch.bfloat16, device=device)
    a2[:, :K], a2[:, K] = a, 1.0
    w2 = torch.zeros(Nn, kp, dtype=torch.bfloat16, device=device)
    w2[:, :K], w2[:, K] = w, b
    lin = N.gemm_epi(a2, w2)
    ref = F.linear(a, w, b).float()
    truth = a.double() @ w.double().t() + b.double()
    d = (lin.float() - ref).abs()
    ulp = torch.maximum(lin.float().abs(), ref.abs()).clamp_min(2 ** -30) * 2 ** -7
    e_got, e_ref = (lin.double() - truth).norm() / truth.norm(), (ref.double() - truth).norm() / truth.norm()
    print(f"bias-column GEMM: differs on {(d > 0).float().mean().item():.4f}, rel-L2 vs fp64 {e_got:.2e} "
          f"(library {e_ref:.2e})")
    assert (d <= ulp * 1.01).all() and (d > 0).float().mean().item() <= 0.05
    assert e_got <= 1.2 * e_ref + 1e-4
    # the GELU epilogue is cp25_gelu on the rounded sum, bit for bit
    assert torch.equal(N.gemm_epi(a2, w2, epilogue=N.EPI_GELU), N.gelu_(lin.clone()))


def test_prepare_context_own_vs_library(device):
    """The whole per-prompt context (crossattn_proj + GELU, per-block k/v projections, k RMSNorm) on the hand-written
    GEMM vs the same steps on the library GEMM (F.linear, computed here as the reference): bf16-rounding-order noise
    only."""
    net = _tiny_net(device)
    p = net.sd
    g = torch.Generator().manual_seed(9)
    emb = torch.randn(2, 512, net.cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16).to(device)
    own = net.prepare_context(emb)
    H, hd = net.cfg.num_heads, net.cfg.head_dim
    ctx = F.linear(emb.reshape(-1, emb.shape[-1]), p["crossattn_proj.0.weight"], p["crossattn_proj.0.bias"])
    N.gelu_(ctx)
    lib_k, lib_v = [], []
    for i in range(net.cfg.num_blocks):
        k = F.linear(ctx, p[f"blocks.{i}.cross_attn.k_proj.weight"])
        N.head_rmsnorm_rope(k, n_rows=ctx.shape[0], B=1, H=H, head_off=0,
                            weight=p[f"blocks.{i}.cross_attn.k_norm.weight"])
        lib_k.append(k)
        lib_v.append(F.linear(ctx, p[f"blocks.{i}.cross_attn.v_proj.weight"]))
    for a, b in zip(own.k + own.v, lib_k + lib_v):
        rel = ((a.float().reshape(-1) - b.float().reshape(-1)).norm() / b.float().norm()).item()
        assert rel <= 4e-3, rel
