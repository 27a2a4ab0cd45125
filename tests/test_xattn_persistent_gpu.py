"""The persistent short-key attention form (text cross-attention) against the per-block form it replaces.

Reference op: the DiT's text cross-attention, minimal_v4_dit.py:1216-1226 -> networks/attention.py:90-181
(softmax(q k^T / sqrt(D)) v over Lk = 512 text tokens). The persistent form (attn_fwd_m16<.., kPersist>, one workgroup
per CU walking a run of query blocks as one K/V tile stream, the next block's Q staged through LDS) does each block's
arithmetic exactly as the per-block form, so the two must be bit-identical (torch.equal) on every shape: ragged key
tiles, the smallest persistent case (2 key tiles), single-block runs, ragged query blocks, many blocks per workgroup,
the DiT's token-major strided views and the full 109 120 x 512 launch. Both are also held to the attention tolerance
against fp32 (4e-3, tests/test_attention_gpu.py).
"""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

TOL = 4e-3
LOG2E = 1.4426950408889634


def _rms_rows(t, w):
    tf = t.float()
    return (tf * torch.rsqrt(tf.pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16)


def _inputs(device, B, H, Lq, Lk, seed, token_major=False):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w = 0.5 + torch.rand(128, generator=g)
    if token_major:  # q as the DiT holds it: [Lq, B, H, D] viewed as [B, Lq, H, D]
        q = _rms_rows(torch.randn(Lq, B, H, 128, generator=g), w).to(device).transpose(0, 1)
    else:
        q = _rms_rows(torch.randn(B, Lq, H, 128, generator=g), w).to(device)
    k = _rms_rows(torch.randn(B, Lk, H, 128, generator=g), w).to(device)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    return q, k, v


def _ref(q, k, v, scale):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    p = torch.softmax(torch.matmul(qf, kf.transpose(-1, -2)) * scale, dim=-1)
    return torch.matmul(p, vf).transpose(1, 2)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


def _both_forms(fn):
    prev = N.attn_cross_select(1)
    try:
        o_p = fn()
        N.attn_cross_select(0)
        o_b = fn()
    finally:
        N.attn_cross_select(prev)
    torch.cuda.synchronize()
    return o_p, o_b


SHAPES = [  # B, H, Lq, Lk
    (2, 4, 5000, 512),   # the DiT's text length, several blocks per workgroup
    (1, 2, 777, 300),    # ragged query block and ragged key tile
    (2, 3, 40, 100),     # one block per (b, h) (fewer blocks than CUs), 2 key tiles (the smallest persistent case)
    (1, 1, 300, 64),     # one key tile: the per-block form runs for both selections
    (2, 8, 20000, 4096), # the largest short-key length
    (1, 16, 2049, 513),  # one key past a tile
]


@pytest.mark.parametrize("B,H,Lq,Lk", SHAPES)
@pytest.mark.parametrize("mode", ["zero", "online_prescaled", "online"])
def test_persistent_equals_per_block(device, B, H, Lq, Lk, mode):
    q, k, v = _inputs(device, B, H, Lq, Lk, 1000 + Lq + Lk, token_major=(Lk == 512))
    scale = 128 ** -0.5
    if mode == "online":
        call = lambda: N.attn_fwd(q, k, v, softmax_scale=scale, n_split=1)
        ref = _ref(q, k, v, scale)
    else:
        qs = (q.float() * (scale * LOG2E)).to(torch.bfloat16)
        bounds = None
        if mode == "zero":
            bounds = (qs.float().norm(dim=-1).max().item() * 1.01, k.float().norm(dim=-1).max().item() * 1.01)
        call = lambda: N.attn_fwd(qs, k, v, prescaled=True, norm_bounds=bounds, n_split=1)
        ref = _ref(qs, k, v, 1.0 / LOG2E)
    o_p, o_b = _both_forms(call)
    e = _rel(o_p, ref)
    print(f"xattn B={B} H={H} Lq={Lq} Lk={Lk} {mode}: persistent vs fp32 {e:.2e}, equal {torch.equal(o_p, o_b)}")
    assert torch.isfinite(o_p.float()).all()
    assert torch.equal(o_p, o_b)
    assert e <= TOL


def test_persistent_full_dit_launch(device):
    """The bench's launch: q token-major [109 120, 2, 16, 128] (the fused layout's stride), 512 text keys."""
    B, H, Lq, Lk = 2, 16, 109120, 512
    g = torch.Generator(device="cpu").manual_seed(7)
    q = torch.randn(Lq, B, H * 128, generator=g).to(device, torch.bfloat16)
    q = torch.nn.functional.normalize(q.view(Lq, B, H, 128).float(), dim=-1).mul(11.3 * 128 ** -0.5 * LOG2E)
    q = q.to(torch.bfloat16).transpose(0, 1)
    k = torch.nn.functional.normalize(torch.randn(B, Lk, H, 128, generator=g), dim=-1).mul(11.3).to(device, torch.bfloat16)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    bounds = (11.3 * 1.01 * 128 ** -0.5 * LOG2E, 11.3 * 1.01)
    o_p, o_b = _both_forms(lambda: N.attn_fwd(q, k, v, prescaled=True, norm_bounds=bounds, n_split=1))
    assert torch.equal(o_p, o_b)
    rows = torch.arange(0, Lq, 997, device=device)
    ref = _ref(q[:, rows], k, v, 1.0 / LOG2E)
    e = _rel(o_p[:, rows], ref)
    print(f"xattn full DiT launch: persistent vs fp32 (sampled rows) {e:.2e}")
    assert e <= TOL


def test_kernel_names(device):
    prev = N.attn_cross_select(1)
    try:
        assert "persistent" in N.attn_kernel_name(512, norm_bounds=(11.0, 11.0), prescaled=True)
        assert "persistent" in N.attn_kernel_name(512, prescaled=True)
        assert "persistent" not in N.attn_kernel_name(64, prescaled=True)       # one key tile
        assert "persistent" not in N.attn_kernel_name(109120, prescaled=True)   # self-attention
        N.attn_cross_select(0)
        assert "persistent" not in N.attn_kernel_name(512, prescaled=True)
    finally:
        N.attn_cross_select(prev)
    with pytest.raises(ValueError):
        N.attn_cross_select(2)
