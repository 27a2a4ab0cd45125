"""Parity of the HIP flash-attention kernel (cp25_attn_fwd) against an fp32 reference of the same op.

Reference op: networks/attention.py:90-181 — q/k/v recast to bf16, softmax(q k^T / sqrt(D)) v.
Oracle here: the same formula in fp32 on the bf16 inputs, output rounded to bf16.
Tolerance: rel-L2 <= 4e-3 and max-abs <= 3e-2. Derivation: every flash-attention kernel the
reference dispatches to (FA2/FA3/cuDNN) rounds the softmax numerator P to bf16 before P.V, which alone
is a ~2^-9/sqrt(3) ~ 1.1e-3 relative error on O, plus bf16 rounding flips of the output itself;
measured 2.2e-3 at Lk = 64 on random data.
"""
import math

import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

TOL = 4e-3


def ref_attention(q, k, v, scale=None):
    # q [B,Lq,H,D] -> fp32 math
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * (scale if scale is not None else q.shape[-1] ** -0.5)
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(torch.bfloat16)


def rel_l2(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize(
    "B,H,Lq,Lk",
    [(1, 1, 32, 64), (2, 3, 300, 77), (1, 2, 256, 512), (2, 2, 1000, 1030), (1, 16, 257, 768), (1, 1, 5, 3)],
)
def test_attn_matches_fp32(device, B, H, Lq, Lk):
    g = torch.Generator(device="cpu").manual_seed(1234 + Lq + Lk)
    q = torch.randn(B, Lq, H, 128, generator=g).to(device, torch.bfloat16)
    k = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    o = N.attn_fwd(q, k, v)
    torch.cuda.synchronize()
    ref = ref_attention(q, k, v)
    assert torch.isfinite(o.float()).all()
    assert rel_l2(o, ref) <= TOL, rel_l2(o, ref)
    assert (o.float() - ref.float()).abs().max().item() <= 3e-2


def test_attn_strided_qkv_buffer(device):
    """q/k/v as views of one fused [L, B, 3, H, 128] projection buffer (the DiT's token-major layout)."""
    L, B, H = 700, 2, 4
    g = torch.Generator(device="cpu").manual_seed(7)
    qkv = torch.randn(L, B, 3, H, 128, generator=g).to(device, torch.bfloat16)
    q = qkv[:, :, 0].transpose(0, 1)  # [B, L, H, D] view
    k = qkv[:, :, 1].transpose(0, 1)
    v = qkv[:, :, 2].transpose(0, 1)
    out = torch.empty(L, B, H, 128, dtype=torch.bfloat16, device=device)
    N.attn_fwd(q, k, v, out=out.transpose(0, 1))
    ref = ref_attention(q.contiguous(), k.contiguous(), v.contiguous())
    assert rel_l2(out.transpose(0, 1), ref) <= TOL


def test_attn_rescale_branch(device):
    """Force the online-softmax running max to jump late (rule 26): a spiked key in the last tile."""
    B, H, Lq, Lk = 1, 2, 256, 640
    g = torch.Generator(device="cpu").manual_seed(3)
    q = torch.randn(B, Lq, H, 128, generator=g)
    k = torch.randn(B, Lk, H, 128, generator=g) * 0.1
    v = torch.randn(B, Lk, H, 128, generator=g)
    k[:, Lk - 5] = q[:, 17] * 3.0  # one key aligned with query 17 in the last tile
    k[:, 100] = -q[:, 40] * 2.0
    q, k, v = (t.to(device, torch.bfloat16) for t in (q, k, v))
    o = N.attn_fwd(q, k, v)
    ref = ref_attention(q, k, v)
    assert rel_l2(o, ref) <= TOL


def test_attn_cross_shape(device):
    """Cross-attention: video tokens against 512 text tokens."""
    B, H, Lq, Lk = 2, 16, 2048, 512
    g = torch.Generator(device="cpu").manual_seed(11)
    q = torch.randn(B, Lq, H, 128, generator=g).to(device, torch.bfloat16)
    k = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    assert rel_l2(N.attn_fwd(q, k, v), ref_attention(q, k, v)) <= TOL


def test_attn_rejects_bad_args(device):
    q = torch.zeros(1, 8, 1, 64, dtype=torch.bfloat16, device=device)
    with pytest.raises(ValueError):
        N.attn_fwd(q, q, q)


@pytest.mark.parametrize("B,H,Lq,Lk,n_split", [(1, 2, 300, 1030, 2), (2, 3, 513, 640, 3), (1, 1, 64, 130, 3),
                                               (2, 2, 256, 4160, 8), (1, 4, 700, 64, 1)])
def test_attn_split_matches_fp32(device, B, H, Lq, Lk, n_split):
    """Key-range split (cp25_attn_fwd_split): fp32 partials + log-sum-exp merge; ragged last range."""
    g = torch.Generator(device="cpu").manual_seed(99 + Lq + n_split)
    q = torch.randn(B, Lq, H, 128, generator=g).to(device, torch.bfloat16)
    k = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    o = N.attn_fwd(q, k, v, n_split=n_split)
    ref = ref_attention(q, k, v)
    assert rel_l2(o, ref) <= TOL, rel_l2(o, ref)
    o1 = N.attn_fwd(q, k, v, n_split=1)
    # split and unsplit differ only by P rounding against different running maxima
    assert rel_l2(o, o1) <= TOL


def test_attn_split_spike_in_one_range(device):
    """A key that dominates one query's softmax lives in the last split only: the merge weights
    (exp2 of the per-range log-sum-exp) must carry it."""
    B, H, Lq, Lk = 1, 1, 256, 1024
    g = torch.Generator(device="cpu").manual_seed(5)
    q = torch.randn(B, Lq, H, 128, generator=g)
    k = torch.randn(B, Lk, H, 128, generator=g) * 0.1
    v = torch.randn(B, Lk, H, 128, generator=g)
    k[:, Lk - 3] = q[:, 9] * 4.0
    q, k, v = (t.to(device, torch.bfloat16) for t in (q, k, v))
    o = N.attn_fwd(q, k, v, n_split=4)
    assert rel_l2(o, ref_attention(q, k, v)) <= TOL


def test_attn_plan_and_bad_split(device):
    assert N.attn_plan(2, 16, 109120, 109120) >= 1
    # a grid far below one workgroup per CU (one query block against long keys) is split
    assert N.attn_plan(1, 1, 256, 109120) > 1
    q = torch.zeros(1, 64, 1, 128, dtype=torch.bfloat16, device=device)
    with pytest.raises(ValueError):
        N.attn_fwd(q, q, q, n_split=2)  # one 64-key tile cannot be split in two


def _rms_rows(t, w):
    """q/k rows as the DiT's q/k RMSNorm leaves them: x / rms(x) * w (bf16)."""
    tf = t.float()
    return (tf * torch.rsqrt(tf.pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16)


def _bounds(q, k):
    return (q.float().norm(dim=-1).max().item(), k.float().norm(dim=-1).max().item())


@pytest.mark.parametrize(
    "B,H,Lq,Lk,n_split",
    [(1, 1, 32, 64, 1), (2, 3, 300, 77, 1), (2, 2, 1000, 1030, 1), (1, 2, 513, 4100, 1), (1, 2, 777, 3000, 3),
     (1, 1, 5, 3, 1)],
)
def test_attn_bounded_shift_matches_fp32(device, B, H, Lq, Lk, n_split):
    """cp25_attn_fwd_bounded: the Cauchy-Schwarz shift |q| max|k| scale replaces the running max
    (softmax shift invariance) — same tolerance vs fp32, and within bf16 rounding of the online form."""
    g = torch.Generator(device="cpu").manual_seed(99 + Lq + Lk)
    w = 0.5 + torch.rand(128, generator=g)
    q = _rms_rows(torch.randn(B, Lq, H, 128, generator=g), w).to(device)
    k = _rms_rows(torch.randn(B, Lk, H, 128, generator=g), w).to(device)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    nb = _bounds(q, k)
    o = N.attn_fwd(q, k, v, n_split=n_split, norm_bounds=nb)
    o_online = N.attn_fwd(q, k, v, n_split=n_split)
    torch.cuda.synchronize()
    ref = ref_attention(q, k, v)
    assert torch.isfinite(o.float()).all()
    assert rel_l2(o, ref) <= TOL, rel_l2(o, ref)
    # P is rounded to bf16 at a different shift in each form: two independent ~2.2e-3 errors (sqrt 2)
    assert rel_l2(o, o_online) <= 1.5 * TOL, rel_l2(o, o_online)


@pytest.mark.parametrize("bound", [48.0, 78.0, 97.5])
def test_attn_bounded_shift_near_cap(device, bound):
    """Score bounds b up to the 98 (log2) cap: the shift max(b - 96, 0) keeps sharp rows right."""
    g = torch.Generator(device="cpu").manual_seed(5)
    B, H, Lq, Lk = 1, 2, 300, 700
    r = (bound * 128 ** 0.5 / 1.4426950408889634) ** 0.5  # |q| = |k| = r -> b = bound (log2 units)
    q = torch.randn(B, Lq, H, 128, generator=g)
    k = torch.randn(B, Lk, H, 128, generator=g)
    q = (q / q.norm(dim=-1, keepdim=True) * r * 0.999).to(device, torch.bfloat16)
    k = (k / k.norm(dim=-1, keepdim=True) * r * 0.999).to(device, torch.bfloat16)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    o = N.attn_fwd(q, k, v, norm_bounds=(r, r))
    torch.cuda.synchronize()
    ref = ref_attention(q, k, v)
    assert torch.isfinite(o.float()).all()
    assert rel_l2(o, ref) <= TOL, rel_l2(o, ref)


def test_attn_bounded_shift_extremes(device):
    """Rows whose every score sits at +b or at -b (b = 78, keys parallel / antiparallel to the query):
    the terms reach 2^60 and 2^-96 and both rows must still average V exactly."""
    g = torch.Generator(device="cpu").manual_seed(11)
    r = (78.0 * 128 ** 0.5 / 1.4426950408889634) ** 0.5
    u = torch.randn(128, generator=g)
    u = u / u.norm() * r * 0.999
    Lq, Lk = 64, 200
    q = torch.randn(1, Lq, 1, 128, generator=g)
    q = q / q.norm(dim=-1, keepdim=True) * r * 0.999
    q[0, 0, 0], q[0, 1, 0] = u, -u
    k = u.expand(1, Lk, 1, 128).clone()
    q, k = q.to(device, torch.bfloat16), k.to(device, torch.bfloat16)
    v = torch.randn(1, Lk, 1, 128, generator=g).to(device, torch.bfloat16)
    o = N.attn_fwd(q, k, v, norm_bounds=(r, r))
    torch.cuda.synchronize()
    mean_v = v.float().mean(1)[0, 0]
    for row in (0, 1):
        assert torch.isfinite(o[0, row, 0].float()).all()
        assert rel_l2(o[0, row, 0], mean_v) <= TOL, (row, rel_l2(o[0, row, 0], mean_v))


def test_attn_bounded_shift_over_cap_is_online(device):
    """Bounds whose shift would exceed the cap select the online-max kernel: bitwise the plain path."""
    g = torch.Generator(device="cpu").manual_seed(6)
    q, k, v = (torch.randn(1, 400, 2, 128, generator=g).to(device, torch.bfloat16) for _ in range(3))
    o = N.attn_fwd(q, k, v, norm_bounds=(1e3, 1e3))
    o_plain = N.attn_fwd(q, k, v)
    torch.cuda.synchronize()
    assert torch.equal(o, o_plain)
    with pytest.raises(ValueError):
        N.attn_fwd(q, k, v, norm_bounds=(-1.0, 1.0))


def test_attn_bounded_shift_violated_bound_is_loud(device):
    """A caller bound far below the real norms overflows the row sum: the guard poisons the row
    (non-finite output) instead of returning a silently wrong one."""
    g = torch.Generator(device="cpu").manual_seed(8)
    u = torch.randn(128, generator=g)
    u = u / u.norm() * 40.0
    q = u.expand(1, 64, 1, 128).contiguous().to(device, torch.bfloat16)
    k = u.expand(1, 128, 1, 128).contiguous().to(device, torch.bfloat16)
    v = torch.randn(1, 128, 1, 128, generator=g).to(device, torch.bfloat16)
    o = N.attn_fwd(q, k, v, norm_bounds=(1.0, 1.0))
    torch.cuda.synchronize()
    assert not torch.isfinite(o.float()).all()


@pytest.mark.parametrize("bounded", [False, True])
def test_attn_full_metric_shape_query_slice(device, bounded):
    """BASELINE config 2's self-attention launch (B 2, H 16, L = Lk = 109 120, RMS-normed q/k as the
    DiT feeds it): 384 query rows checked against fp32 attention over all 109 120 keys, and
    V = const -> O = const for every row (the normalised weights sum to 1)."""
    L, B, H = 109120, 2, 16
    g = torch.Generator(device=device).manual_seed(3)
    w = 0.5 + torch.rand(128, device=device, generator=g)
    q = _rms_rows(torch.randn(B, L, H, 128, device=device, generator=g), w)
    k = _rms_rows(torch.randn(B, L, H, 128, device=device, generator=g), w)
    v = torch.randn(B, L, H, 128, device=device, generator=g).to(torch.bfloat16)
    nb = _bounds(q, k) if bounded else None
    o = N.attn_fwd(q, k, v, norm_bounds=nb)
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(4))[:384].to(device)
    err = []
    for b in range(B):
        for h in range(H):
            s = (q[b, rows, h].float() @ k[b, :, h].float().t()) * 128 ** -0.5
            ref = torch.softmax(s, -1) @ v[b, :, h].float()
            err.append(((o[b, rows, h].float() - ref).norm() / ref.norm()).item())
    assert max(err) <= TOL, max(err)
    vc = torch.full_like(v, 0.75)
    oc = N.attn_fwd(q, k, vc, norm_bounds=nb)
    torch.cuda.synchronize()
    assert ((oc.float() - 0.75).abs() <= 0.75 * 2 ** -7).all()
