"""The gated fixed-shift / online-max attention pair (cp25_attn_fwd_prescaled_kslots) and its data-tight key bound
(cp25_head_rmsnorm_rope_nmax).

Reference op: networks/attention.py:90-181 after the q/k RMSNorms of minimal_v4_dit.py:355-358 (learnable weights:
a trained checkpoint's max|w| puts the weight-based bound sqrt(128) max|w_q| max|w_k| past the zero-shift window).
The k RMSNorm kernel measures the max |k row| it writes; with it a 256-query block whose bound max|q_row| max|k|
is <= 110 runs the fixed-shift loop on that measured bound (round 6; it was the zero shift up to 96), any other block
the online max. Checks: the measured bound equals the true max row norm; every block's output is bit-identical to the
mode it was routed to (fixed shift / online max, each launched on its own); attention tolerance vs fp32 (4e-3, tests/test_attention_gpu.py).
"""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu

LOG2E = 1.4426950408889634
TOL = 4e-3


def _ref(q, k, v, scale):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    p = torch.softmax(torch.matmul(qf, kf.transpose(-1, -2)) * scale, dim=-1)
    return torch.matmul(p, vf).transpose(1, 2)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_head_rmsnorm_rope_norm_max(device):
    """The 64 slots' max is the max |row| of the written bf16 result (over rows and heads), with or without RoPE."""
    g = torch.Generator(device="cpu").manual_seed(3)
    n_tok, B, H, D = 777, 2, 4, 4 * 128
    buf = torch.randn(n_tok * B, 3 * D, generator=g).to(device, torch.bfloat16)
    w = (0.5 + 2.5 * torch.rand(128, generator=g)).to(device, torch.bfloat16)
    cos = torch.rand(n_tok, 64, generator=g).to(device)
    sin = (1 - cos ** 2).sqrt()
    slots = torch.zeros((64, 32), dtype=torch.float32, device=device)
    N.head_rmsnorm_rope(buf, n_rows=n_tok * B, B=B, H=H, head_off=D, weight=w, cos=cos, sin=sin, norm_max=slots)
    torch.cuda.synchronize()
    true = buf[:, D:2 * D].float().view(-1, H, 128).norm(dim=-1).max().item()
    got = slots[:, 0].max().item()
    assert (slots[:, 1:] == 0).all()
    print(f"norm max: slots {got:.6f} true {true:.6f}")
    assert abs(got - true) <= 1e-5 * true
    assert (slots >= 0).all()


def _qk(device, B, H, L, Lk, wq, wk, seed, big_rows=None):
    g = torch.Generator(device="cpu").manual_seed(seed)

    def rms(t, w):
        return (t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16)

    q = rms(torch.randn(B, L, H, 128, generator=g), wq)
    if big_rows is not None:  # rows scaled up: their blocks' bound leaves the zero-shift window
        q[:, big_rows] = (q[:, big_rows].float() * 3.0).to(torch.bfloat16)
    k = rms(torch.randn(B, Lk, H, 128, generator=g), wk)
    v = torch.randn(B, Lk, H, 128, generator=g).to(torch.bfloat16)
    c = 128 ** -0.5 * LOG2E
    qs = (q.float() * c).to(torch.bfloat16)
    return qs.to(device), k.to(device), v.to(device)


@pytest.mark.parametrize("B,H,L,mixed", [(2, 4, 3000, False), (1, 4, 2000, True), (2, 2, 777, True)])
def test_gated_pair_routes_blocks_bit_identically(device, B, H, L, mixed):
    g = torch.Generator(device="cpu").manual_seed(11)
    wq, wk = 0.5 + 2.5 * torch.rand(128, generator=g), 0.5 + 2.5 * torch.rand(128, generator=g)
    big = torch.arange(300, 420) if mixed else None  # rows of the 2nd query block (256 .. 511)
    qs, k, v = _qk(device, B, H, L, L, wq, wk, 5 + L, big)
    # weight-based bounds (the DiT's refresh_norm_bounds): product past 96
    qb, kb = 128 ** 0.5 * float(wq.max()) * 1.02 * 128 ** -0.5 * LOG2E, 128 ** 0.5 * float(wk.max()) * 1.02
    assert qb * kb > 96.0
    slots = torch.zeros((64, 32), dtype=torch.float32, device=device)
    slots[3, 0] = k.float().norm(dim=-1).max()  # what head_rmsnorm_rope_nmax would write (any slot)
    o = N.attn_fwd(qs, k, v, prescaled=True, norm_bounds=(qb, kb), k_norm_slots=slots, n_split=1)
    # the two modes on their own: the fixed shift with the measured key bound x 1.001 (fp32, as the kernel forms it;
    # a q bound that makes the product 97 selects the fixed mode) and the online max (no bounds)
    kd = (slots[3:4, 0] * torch.tensor([1.001], dtype=torch.float32, device=device)).item()
    o_fixed = N.attn_fwd(qs, k, v, prescaled=True, norm_bounds=(97.0 / kd, kd), n_split=1)
    o_onl = N.attn_fwd(qs, k, v, prescaled=True, n_split=1)
    torch.cuda.synchronize()
    kmax = k.float().norm(dim=-1).max().item()
    nblk = (L + 255) // 256
    n_fixed = 0
    for b in range(B):
        for h in range(H):
            for j in range(nblk):
                r = slice(256 * j, min(256 * (j + 1), L))
                qmax = qs[b, r, h].float().norm(dim=-1).max().item()
                fixed_ok = qmax * kmax * 1.001 <= 110.0  # attn_common.h kGateFixed
                n_fixed += fixed_ok
                want = o_fixed if fixed_ok else o_onl
                assert torch.equal(o[b, r, h], want[b, r, h]), (b, h, j, fixed_ok)
    e = _rel(o, _ref(qs, k, v, 1.0 / LOG2E))
    print(f"gated B={B} H={H} L={L} mixed={mixed}: {n_fixed}/{B * H * nblk} blocks fixed-shift, vs fp32 {e:.2e}")
    assert e <= TOL
    assert n_fixed > 0
    if not mixed:
        assert n_fixed == B * H * nblk
    assert torch.isfinite(o.float()).all()


def test_gated_pair_without_slots_is_online(device):
    """Unwritten (zero) slots are no bound: every block runs the online max."""
    qs, k, v = _qk(device, 1, 2, 600, 600, torch.full((128,), 3.0), torch.full((128,), 3.0), 1)
    slots = torch.zeros((64, 32), dtype=torch.float32, device=device)
    o = N.attn_fwd(qs, k, v, prescaled=True, norm_bounds=(40.0, 40.0), k_norm_slots=slots, n_split=1)
    o_onl = N.attn_fwd(qs, k, v, prescaled=True, n_split=1)
    torch.cuda.synchronize()
    assert torch.equal(o, o_onl)


def test_gated_kernel_name(device):
    assert "gated" in N.attn_kernel_name(109120, norm_bounds=(4.4, 34.6), prescaled=2)
    # no gate where the weight bounds suffice: long keys take the fixed shift up to a product of 110 (whole bound to 63),
    # short keys the zero shift up to 96
    assert "fixed shift" in N.attn_kernel_name(109120, norm_bounds=(1.5, 11.6), prescaled=2)
    assert "fixed shift" in N.attn_kernel_name(109120, norm_bounds=(8.5, 12.5), prescaled=2)
    assert "gated" in N.attn_kernel_name(109120, norm_bounds=(9.0, 12.5), prescaled=2)
    assert "zero shift" in N.attn_kernel_name(512, norm_bounds=(7.0, 11.6), prescaled=2)
