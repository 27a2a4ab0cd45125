"""attn_fwd_m16: the bounded-shift / prescaled self- and cross-attention on v_mfma_f32_16x16x32_bf16
(CP25_ATTN_MFMA=16) vs fp32 attention on the same bf16 q / k / v, and vs the 32x32x16 kernel it replaces.

Reference op: networks/attention.py:90-181 (softmax(q k^T / sqrt(D)) v, bf16 operands). Same tolerance as
tests/test_attention_gpu.py (rel-L2 <= 4e-3 vs fp32: P rounded to bf16 before P.V, bf16 output). The two
MFMA shapes sum the same products in a different order, so the forms agree to fp32 accumulation noise plus
bf16 rounding flips of P and of O (bound 1.5 x TOL, as two independent roundings of the same answer).
The switch is read per launch, so each test sets it with monkeypatch.
"""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

TOL = 4e-3
LOG2E = 1.4426950408889634


def ref_attention(q, k, v, scale):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    p = torch.softmax(torch.matmul(qf, kf.transpose(-1, -2)) * scale, dim=-1)
    return torch.matmul(p, vf).transpose(1, 2).to(torch.bfloat16)


def rel_l2(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _rms_rows(t, w):
    tf = t.float()
    return (tf * torch.rsqrt(tf.pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16)


def _inputs(device, B, H, Lq, Lk, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w = 0.5 + torch.rand(128, generator=g)
    q = _rms_rows(torch.randn(B, Lq, H, 128, generator=g), w).to(device)
    k = _rms_rows(torch.randn(B, Lk, H, 128, generator=g), w).to(device)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    return q, k, v


def _run(monkeypatch, shape, fn):
    monkeypatch.setenv("CP25_ATTN_MFMA", shape)
    o = fn()
    torch.cuda.synchronize()
    return o


@pytest.mark.parametrize(
    "B,H,Lq,Lk,n_split",
    [(1, 1, 32, 64, 1), (2, 3, 300, 77, 1), (2, 2, 1000, 1030, 1), (1, 2, 513, 4100, 1), (1, 2, 777, 3000, 3),
     (1, 1, 5, 3, 1), (1, 2, 64, 4097, 5), (2, 4, 4800, 512, 1)],
)
@pytest.mark.parametrize("prescaled", [False, True])
def test_m16_matches_fp32(device, monkeypatch, B, H, Lq, Lk, n_split, prescaled):
    """Ragged query blocks and key tiles, key-range splits, cross-attention lengths (Lk <= 4096 selects the
    cross-attention instantiation), both forms the DiT launches."""
    q, k, v = _inputs(device, B, H, Lq, Lk, 321 + Lq + Lk)
    scale = 128 ** -0.5
    qn, kn = q.float().norm(dim=-1).max().item(), k.float().norm(dim=-1).max().item()
    if prescaled:
        c = scale * LOG2E
        qs = (q.float() * c).to(torch.bfloat16)
        nb = (qn * c * 1.01, kn)
        args = dict(norm_bounds=nb, prescaled=True, n_split=n_split)
        ref = ref_attention(qs, k, v, 1.0 / LOG2E)
        qin = qs
    else:
        args = dict(norm_bounds=(qn, kn), n_split=n_split)
        ref = ref_attention(q, k, v, scale)
        qin = q
    o16 = _run(monkeypatch, "16", lambda: N.attn_fwd(qin, k, v, **args))
    o32 = _run(monkeypatch, "32", lambda: N.attn_fwd(qin, k, v, **args))
    assert torch.isfinite(o16.float()).all()
    e16, e32, e = rel_l2(o16, ref), rel_l2(o32, ref), rel_l2(o16, o32)
    print(f"m16 B={B} H={H} Lq={Lq} Lk={Lk} split={n_split} prescaled={prescaled}: vs fp32 {e16:.2e} "
          f"(32x32x16 kernel {e32:.2e}), m16 vs 32x32x16 {e:.2e}")
    assert e16 <= TOL, e16
    assert e <= 1.5 * TOL, e


def test_m16_strided_token_major_views(device, monkeypatch):
    """q / k / v as views of the DiT's fused token-major [L, B, 3, H, 128] buffer, output into a strided view."""
    L, B, H = 700, 2, 4
    g = torch.Generator(device="cpu").manual_seed(17)
    w = 0.5 + torch.rand(128, generator=g)
    qkv = _rms_rows(torch.randn(L, B, 3, H, 128, generator=g), w).to(device)
    q, k, v = (qkv[:, :, i].transpose(0, 1) for i in range(3))
    out = torch.empty(L, B, H, 128, device=device, dtype=torch.bfloat16)
    nb = (q.float().norm(dim=-1).max().item(), k.float().norm(dim=-1).max().item())
    _run(monkeypatch, "16", lambda: N.attn_fwd(q, k, v, out=out.transpose(0, 1), norm_bounds=nb))
    ref = ref_attention(q, k, v, 128 ** -0.5)
    assert rel_l2(out.transpose(0, 1), ref) <= TOL


def test_m16_extremes_and_guard(device, monkeypatch):
    """Rows whose every score sits at +b or -b (b = 78 log2 units: terms 2^60 and 2^-96) still average V; a norm
    bound far below the real norms poisons the rows (non-finite) instead of a silent wrong answer."""
    g = torch.Generator(device="cpu").manual_seed(11)
    r = (78.0 * 128 ** 0.5 / LOG2E) ** 0.5
    u = torch.randn(128, generator=g)
    u = u / u.norm() * r * 0.999
    q = torch.randn(1, 64, 1, 128, generator=g)
    q = q / q.norm(dim=-1, keepdim=True) * r * 0.999
    q[0, 0, 0], q[0, 1, 0] = u, -u
    k = u.expand(1, 200, 1, 128).clone()
    q, k = q.to(device, torch.bfloat16), k.to(device, torch.bfloat16)
    v = torch.randn(1, 200, 1, 128, generator=g).to(device, torch.bfloat16)
    o = _run(monkeypatch, "16", lambda: N.attn_fwd(q, k, v, norm_bounds=(r, r)))
    mean_v = v.float().mean(1)[0, 0]
    for row in (0, 1):
        assert rel_l2(o[0, row, 0], mean_v) <= TOL
    u2 = u / u.norm() * 40.0
    qb = u2.expand(1, 64, 1, 128).contiguous().to(device, torch.bfloat16)
    kb = u2.expand(1, 128, 1, 128).contiguous().to(device, torch.bfloat16)
    vb = torch.randn(1, 128, 1, 128, generator=g).to(device, torch.bfloat16)
    ob = _run(monkeypatch, "16", lambda: N.attn_fwd(qb, kb, vb, norm_bounds=(1.0, 1.0)))
    assert not torch.isfinite(ob.float()).all()


def test_m16_full_metric_shape_query_slice(device, monkeypatch):
    """BASELINE config 2's self-attention launch (B 2, H 16, L = 109 120, prescaled as the DiT runs it): 384 query
    rows vs fp32 over all keys, and V = const -> O = const for every row."""
    L, B, H = 109120, 2, 16
    g = torch.Generator(device=device).manual_seed(3)
    w = 0.5 + torch.rand(128, device=device, generator=g)
    q = _rms_rows(torch.randn(B, L, H, 128, device=device, generator=g), w)
    k = _rms_rows(torch.randn(B, L, H, 128, device=device, generator=g), w)
    v = torch.randn(B, L, H, 128, device=device, generator=g).to(torch.bfloat16)
    c = 128 ** -0.5 * LOG2E
    qs = (q.float() * c).to(torch.bfloat16)
    nb = (qs.float().norm(dim=-1).max().item() * 1.01, k.float().norm(dim=-1).max().item())
    o = _run(monkeypatch, "16", lambda: N.attn_fwd(qs, k, v, norm_bounds=nb, prescaled=True))
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(4))[:384].to(device)
    err = []
    for b in range(B):
        for h in range(H):
            s = (qs[b, rows, h].float() @ k[b, :, h].float().t()) / LOG2E
            ref = torch.softmax(s, -1) @ v[b, :, h].float()
            err.append(((o[b, rows, h].float() - ref).norm() / ref.norm()).item())
    assert max(err) <= TOL, max(err)
    oc = _run(monkeypatch, "16", lambda: N.attn_fwd(qs, k, torch.full_like(v, 0.75), norm_bounds=nb, prescaled=True))
    assert ((oc.float() - 0.75).abs() <= 0.75 * 2 ** -7).all()


def _vt_reference(v):
    """torch restatement of cp25_cast_v_bf16t: [B][H][tile][128 d][64 p], p = 32 ks + 8 g + j holding key
    32 ks + 16 (j >> 2) + 4 g + (j & 3) of the tile, zero past L."""
    B, L, H, D = v.shape
    nt = (L + 63) // 64
    vp = torch.zeros(B, nt * 64, H, D, dtype=v.dtype, device=v.device)
    vp[:, :L] = v
    p = torch.arange(64)
    key = 32 * (p >> 5) + 16 * ((p & 7) >> 2) + 4 * ((p >> 3) & 3) + (p & 3)
    t = vp.view(B, nt, 64, H, D)[:, :, key.to(v.device)]  # [B, nt, 64 p, H, D]
    return t.permute(0, 3, 1, 4, 2).contiguous().view(-1)  # [B, H, nt, D, 64 p]


@pytest.mark.parametrize("L", [64, 1000, 4097])
def test_v_bf16t_layout_exact(device, L):
    g = torch.Generator(device="cpu").manual_seed(L)
    qkv = torch.randn(L, 2, 3, 4, 128, generator=g).to(device, torch.bfloat16)
    v = qkv[:, :, 2].transpose(0, 1)  # strided [B, L, H, D] view of a token-major buffer
    vt = N.cast_v_bf16t(v)
    torch.cuda.synchronize()
    assert torch.equal(vt, _vt_reference(v))


@pytest.mark.parametrize("B,H,Lq,Lk,n_split", [(1, 1, 32, 64, 1), (2, 3, 300, 77, 1), (2, 2, 1000, 1030, 1),
                                               (1, 2, 777, 3000, 3), (1, 2, 64, 4097, 5), (2, 4, 4800, 512, 1),
                                               (1, 1, 5, 3, 1)])
def test_m16_vt_bit_identical(device, monkeypatch, B, H, Lq, Lk, n_split):
    """cp25_attn_fwd_prescaled_vt (V^T tiles, one ds_read_b128 per P.V operand) = cp25_attn_fwd_prescaled on the
    16x16x32 kernel bit for bit: the same operand values in the same k order."""
    q, k, v = _inputs(device, B, H, Lq, Lk, 77 + Lq + Lk)
    c = 128 ** -0.5 * LOG2E
    qs = (q.float() * c).to(torch.bfloat16)
    nb = (qs.float().norm(dim=-1).max().item() * 1.01, k.float().norm(dim=-1).max().item())
    vt = N.cast_v_bf16t(v)
    o_vt = _run(monkeypatch, "16", lambda: N.attn_fwd(qs, k, v, norm_bounds=nb, prescaled=True, n_split=n_split,
                                                      v_t=vt))
    o = _run(monkeypatch, "16", lambda: N.attn_fwd(qs, k, v, norm_bounds=nb, prescaled=True, n_split=n_split))
    assert torch.equal(o_vt, o)
