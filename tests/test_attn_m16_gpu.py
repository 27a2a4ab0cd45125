"""attn_fwd_m16 (every bf16 attention form) vs fp32 attention on the same bf16 q / k / v, in each of its three
softmax-shift modes, and the modes against each other.

Reference op: networks/attention.py:90-181 (softmax(q k^T / sqrt(D)) v, bf16 operands). Same tolerance as
tests/test_attention_gpu.py (rel-L2 <= 4e-3 vs fp32: P rounded to bf16 before P.V, bf16 output). The modes differ
only in the shift at which P is rounded to bf16, so two modes agree within two independent roundings (1.5 x TOL).
Modes (the library picks one from the norm bounds, attn_fwd.hip):
  fixed  norm bounds with max|q| max|k| <= 98 (log2 units): per-row shift max(|q_row| max|k| - 96, 0);
  zero   pre-scaled q and bound product <= 96: no shift at all (the round-2 prescaled kernel);
  online no bounds or a larger product: the row max of tile 0, moved up lazily (> 24 above the shift).
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


def _inputs(device, B, H, Lq, Lk, seed, wmax=1.5):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w = 0.5 + (wmax - 0.5) * torch.rand(128, generator=g)
    q = _rms_rows(torch.randn(B, Lq, H, 128, generator=g), w).to(device)
    k = _rms_rows(torch.randn(B, Lk, H, 128, generator=g), w).to(device)
    v = torch.randn(B, Lk, H, 128, generator=g).to(device, torch.bfloat16)
    return q, k, v


SHAPES = [(1, 1, 32, 64, 1), (2, 3, 300, 77, 1), (2, 2, 1000, 1030, 1), (1, 2, 513, 4100, 1), (1, 2, 777, 3000, 3),
          (1, 1, 5, 3, 1), (1, 2, 64, 4097, 5), (2, 4, 4800, 512, 1)]


@pytest.mark.parametrize("B,H,Lq,Lk,n_split", SHAPES)
@pytest.mark.parametrize("prescaled", [False, True])
def test_m16_modes_match_fp32(device, B, H, Lq, Lk, n_split, prescaled):
    """Ragged query blocks and key tiles, key-range splits, cross-attention lengths (Lk <= 4096 selects the
    cross-attention instantiation): fixed / zero-shift / online modes vs fp32 and vs each other."""
    q, k, v = _inputs(device, B, H, Lq, Lk, 321 + Lq + Lk)
    scale = 128 ** -0.5
    qn, kn = q.float().norm(dim=-1).max().item(), k.float().norm(dim=-1).max().item()
    if prescaled:
        c = scale * LOG2E
        qin = (q.float() * c).to(torch.bfloat16)
        ref = ref_attention(qin, k, v, 1.0 / LOG2E)
        base = dict(prescaled=True, n_split=n_split)
        qb = qin.float().norm(dim=-1).max().item() * 1.01
        # the data's bounds (product <= 63: the whole-bound fixed shift for long keys, the zero shift for short ones),
        # zero shift (product 80: inflated q bound), fixed shift (product in (96, 98]), online
        modes = {"tight": dict(base, norm_bounds=(qb, kn)), "zero": dict(base, norm_bounds=(max(qb, 80.0 / kn), kn)),
                 "fixed": dict(base, norm_bounds=(97.0 / kn, kn)), "online": dict(base)}
        assert qb * kn <= 63.0
        exp = "fixed shift" if Lk > 4096 else "zero shift"
        assert exp in N.attn_kernel_name(Lk, norm_bounds=(qb, kn), prescaled=True)
        assert exp in N.attn_kernel_name(Lk, norm_bounds=(max(qb, 80.0 / kn), kn), prescaled=True)  # to 110 / 96
    else:
        qin = q
        ref = ref_attention(q, k, v, scale)
        base = dict(n_split=n_split)
        modes = {"fixed": dict(base, norm_bounds=(qn, kn)), "online": dict(base)}
    outs = {m: N.attn_fwd(qin, k, v, **kw) for m, kw in modes.items()}
    torch.cuda.synchronize()
    errs = {m: rel_l2(o, ref) for m, o in outs.items()}
    print(f"m16 B={B} H={H} Lq={Lq} Lk={Lk} split={n_split} prescaled={prescaled}: vs fp32 "
          + ", ".join(f"{m} {e:.2e}" for m, e in errs.items()))
    for m, o in outs.items():
        assert torch.isfinite(o.float()).all(), m
        assert errs[m] <= TOL, (m, errs[m])
        assert rel_l2(o, outs["online"]) <= 1.5 * TOL, m


def test_m16_strided_token_major_views(device):
    """q / k / v as views of the DiT's fused token-major [L, B, 3, H, 128] buffer, output into a strided view."""
    L, B, H = 700, 2, 4
    g = torch.Generator(device="cpu").manual_seed(17)
    w = 0.5 + torch.rand(128, generator=g)
    qkv = _rms_rows(torch.randn(L, B, 3, H, 128, generator=g), w).to(device)
    q, k, v = (qkv[:, :, i].transpose(0, 1) for i in range(3))
    ref = ref_attention(q, k, v, 128 ** -0.5)
    nb = (q.float().norm(dim=-1).max().item(), k.float().norm(dim=-1).max().item())
    for kw in (dict(norm_bounds=nb), dict()):
        out = torch.empty(L, B, H, 128, device=device, dtype=torch.bfloat16)
        N.attn_fwd(q, k, v, out=out.transpose(0, 1), **kw)
        assert rel_l2(out.transpose(0, 1), ref) <= TOL


@pytest.mark.parametrize("bound", [78.0, 97.5])
def test_m16_fixed_extremes_and_guard(device, bound):
    """Fixed mode: rows whose every score sits at +b or -b (b = 78: terms 2^78 and 2^-78, no shift; b = 97.5: shift
    1.5, terms 2^96 and 2^-99) still average V; a norm bound far below the real norms poisons the rows (non-finite)
    instead of a silent wrong answer."""
    g = torch.Generator(device="cpu").manual_seed(11)
    r = (bound * 128 ** 0.5 / LOG2E) ** 0.5
    u = torch.randn(128, generator=g)
    u = u / u.norm() * r * 0.999
    q = torch.randn(1, 64, 1, 128, generator=g)
    q = q / q.norm(dim=-1, keepdim=True) * r * 0.999
    q[0, 0, 0], q[0, 1, 0] = u, -u
    k = u.expand(1, 200, 1, 128).clone()
    q, k = q.to(device, torch.bfloat16), k.to(device, torch.bfloat16)
    v = torch.randn(1, 200, 1, 128, generator=g).to(device, torch.bfloat16)
    o = N.attn_fwd(q, k, v, norm_bounds=(r, r))
    mean_v = v.float().mean(1)[0, 0]
    for row in (0, 1):
        assert rel_l2(o[0, row, 0], mean_v) <= TOL
    u2 = u / u.norm() * 40.0
    qb = u2.expand(1, 64, 1, 128).contiguous().to(device, torch.bfloat16)
    kb = u2.expand(1, 128, 1, 128).contiguous().to(device, torch.bfloat16)
    vb = torch.randn(1, 128, 1, 128, generator=g).to(device, torch.bfloat16)
    ob = N.attn_fwd(qb, kb, vb, norm_bounds=(1.0, 1.0))
    torch.cuda.synchronize()
    assert not torch.isfinite(ob.float()).all()


@pytest.mark.parametrize("prescaled", [False, True])
def test_m16_online_any_range(device, prescaled):
    """Online mode where no fixed shift exists: scores at +-400 log2 units (rows whose every score is -400 would
    underflow any fixed window), a late spike 300 above a row's earlier max (rescale far past the lazy threshold),
    and a spike in the last ragged tile; all against fp32."""
    g = torch.Generator(device="cpu").manual_seed(21)
    Lq, Lk = 300, 1000
    r = (400.0 * 128 ** 0.5 / LOG2E) ** 0.5
    u = torch.randn(128, generator=g)
    u = u / u.norm()
    q = torch.randn(1, Lq, 2, 128, generator=g)
    q = q / q.norm(dim=-1, keepdim=True) * r
    k = torch.randn(1, Lk, 2, 128, generator=g) * 0.05
    k[0, :, 0] = -u * r        # head 0: every key antiparallel to query 0 (all its scores -400)
    q[0, 0, 0] = u * r
    k[0, Lk - 7, 1] = q[0, 5, 1] * 0.9  # head 1: a late spike for query 5 (score ~ +360) in the ragged tile
    k[0, 70, 1] = q[0, 9, 1] * 0.3      # and an earlier moderate one for query 9
    v = torch.randn(1, Lk, 2, 128, generator=g)
    q, k, v = (t.to(device, torch.bfloat16) for t in (q, k, v))
    scale = 128 ** -0.5
    if prescaled:
        qin = (q.float() * scale * LOG2E).to(torch.bfloat16)
        o = N.attn_fwd(qin, k, v, prescaled=True)
        ref = ref_attention(qin, k, v, 1.0 / LOG2E)
    else:
        o = N.attn_fwd(q, k, v)
        ref = ref_attention(q, k, v, scale)
    torch.cuda.synchronize()
    assert torch.isfinite(o.float()).all()
    assert rel_l2(o, ref) <= TOL, rel_l2(o, ref)
    assert rel_l2(o[0, 0, 0], ref[0, 0, 0]) <= TOL
    assert rel_l2(o[0, 5, 1], ref[0, 5, 1]) <= TOL


def test_m16_online_split_merge(device):
    """Online partials of a key-range split carry their own shifts into the log-sum-exp merge."""
    q, k, v = _inputs(device, 1, 2, 513, 3000, 5, wmax=3.0)
    q = (q.float() * 3.0).to(torch.bfloat16)  # sharp rows
    ref = ref_attention(q, k, v, 128 ** -0.5)
    for s in (1, 3, 8):
        o = N.attn_fwd(q, k, v, n_split=s)
        assert rel_l2(o, ref) <= TOL, (s, rel_l2(o, ref))


def test_m16_full_metric_shape_query_slice(device):
    """BASELINE config 2's self-attention launch (B 2, H 16, L = 109 120, prescaled as the DiT runs it) in the
    zero-shift mode (unit norm weights) and the online mode (trained-size weights): 384 query rows vs fp32 over all
    keys, and V = const -> O = const for every row."""
    L, B, H = 109120, 2, 16
    g = torch.Generator(device=device).manual_seed(3)
    c = 128 ** -0.5 * LOG2E
    for wlo, whi, nb_given in ((1.0, 1.0, True), (0.5, 3.0, False)):
        w = wlo + (whi - wlo) * torch.rand(128, device=device, generator=g)
        q = _rms_rows(torch.randn(B, L, H, 128, device=device, generator=g), w)
        k = _rms_rows(torch.randn(B, L, H, 128, device=device, generator=g), w)
        v = torch.randn(B, L, H, 128, device=device, generator=g).to(torch.bfloat16)
        qs = (q.float() * c).to(torch.bfloat16)
        del q
        nb = (qs.float().norm(dim=-1).max().item() * 1.01, k.float().norm(dim=-1).max().item()) if nb_given else None
        o = N.attn_fwd(qs, k, v, norm_bounds=nb, prescaled=True)
        rows = torch.randperm(L, generator=torch.Generator().manual_seed(4))[:384].to(device)
        err = []
        for b in range(B):
            for h in range(H):
                s = (qs[b, rows, h].float() @ k[b, :, h].float().t()) / LOG2E
                ref = torch.softmax(s, -1) @ v[b, :, h].float()
                err.append(((o[b, rows, h].float() - ref).norm() / ref.norm()).item())
        print(f"metric shape, norm weights in [{wlo}, {whi}] ({'fixed/zero' if nb_given else 'online'}): "
              f"max rel-L2 {max(err):.2e}")
        assert max(err) <= TOL, max(err)
        oc = N.attn_fwd(qs, k, torch.full_like(v, 0.75), norm_bounds=nb, prescaled=True)
        torch.cuda.synchronize()
        assert ((oc.float() - 0.75).abs() <= 0.75 * 2 ** -7).all()
        del o, oc, qs, k, v


@pytest.mark.parametrize("Lk,k0,kb,form", [(163840, 11.984375, 12.0, "fixed shift"), (163840, 13.75, 13.75, "fixed shift"),
                                            (4096, 11.984375, 12.0, "zero shift")])
def test_m16_zero_shift_top_of_window_long_keys(device, Lk, k0, kb, form):
    """The windows' headroom: every score of every row at the top of the window over 163 840 keys (> config 4's
    163 800), |v| up to ~400. Long keys take the fixed shift (round 6) up to a bound product of 110 (attn_common.h
    kGateFixed): scores 95.9 and 110 are shifted by floor(126 - b_row) = 30 / 16, so P = 2^65.9 / 2^94 and O stays inside
    fp32; the zero shift (attn_fwd.hip kTop = 96, short keys here) leaves P = 2^95.9 (the row sum 2^107, O ~2^116 over
    4096 keys; the window holds while |v| Lk < 2^32). All terms equal, so O = mean(v) exactly up to the bf16 output
    rounding."""
    Lq = 256
    g = torch.Generator(device="cpu").manual_seed(13)
    q = torch.zeros(1, Lq, 1, 128)
    k = torch.zeros(1, Lk, 1, 128)
    q[..., 0], k[..., 0] = 8.0, k0  # bf16-exact; pre-scaled score 95.875 / 110 (log2 units)
    v = (torch.randn(1, Lk, 1, 128, generator=g) * 100.0).to(device, torch.bfloat16)
    q, k = q.to(device, torch.bfloat16), k.to(device, torch.bfloat16)
    assert form in N.attn_kernel_name(Lk, None, (8.0, kb), True)
    o = N.attn_fwd(q, k, v, norm_bounds=(8.0, kb), prescaled=True)
    torch.cuda.synchronize()
    assert torch.isfinite(o.float()).all()
    mean_v = v.float().mean(1)[0, 0]
    assert rel_l2(o[0, :, 0], mean_v.expand(Lq, 128)) <= 2 ** -8


@pytest.mark.parametrize("sign", [1.0, -1.0])
@pytest.mark.parametrize("k0", [12.5, 3.40625])
def test_m16_whole_bound_shift_edges(device, sign, k0):
    """The fixed shift of long-key launches (round 6: each row shifted by floor(min(b_row + 60, 126 - b_row)),
    attn_common.h kPDrop): every score at +b (the top) or at -b (the bottom) over 8192 keys. b = 62.5: shift 63, P =
    2^-0.5 / 2^-125.5 (still a normal bf16 / fp32); b = 17.03 (the unit weights' range): shift 77, P = 2^-60 / 2^-94.
    All terms equal, so O = mean(v) up to the bf16 output rounding."""
    Lq, Lk = 256, 8192
    g = torch.Generator(device="cpu").manual_seed(14)
    q = torch.zeros(1, Lq, 1, 128)
    k = torch.zeros(1, Lk, 1, 128)
    q[..., 0], k[..., 0] = 5.0, sign * k0  # bf16-exact; pre-scaled score +-62.5 / +-17.03 (log2 units)
    v = (torch.randn(1, Lk, 1, 128, generator=g) * 10.0).to(device, torch.bfloat16)
    q, k = q.to(device, torch.bfloat16), k.to(device, torch.bfloat16)
    assert N.attn_kernel_name(Lk, None, (5.0, k0), True).endswith("fixed shift>")
    o = N.attn_fwd(q, k, v, norm_bounds=(5.0, k0), prescaled=True)
    torch.cuda.synchronize()
    assert torch.isfinite(o.float()).all()
    mean_v = v.float().mean(1)[0, 0]
    assert rel_l2(o[0, :, 0], mean_v.expand(Lq, 128)) <= 2 ** -8


@pytest.mark.parametrize("prescaled", [False, True])
def test_m16_tail_split(device, prescaled):
    """The last, partial round of an unsplit launch as a tail split (cp25_attn_tail_workspace_bytes): a CP = 8 lane's
    shape (B 1, H 16, 13 640 queries: 864 = 3 x 256 + 96 workgroups) with 32 768 keys. The first 768 query blocks run in
    the main launch, bit-identical to the whole unsplit launch; the last 96 (head 14 from block 12, and head 15) as
    key-range splits merged into o, within rounding of it and as close to fp32 (rows of both tail segments)."""
    B, H, Lq, Lk = 1, 16, 13640, 32768
    lib = N.load_library()
    assert lib.cp25_attn_tail_workspace_bytes(B, H, Lq, Lk) > 0 and N.attn_plan(B, H, Lq, Lk) == 1
    q, k, v = _inputs(device, B, H, Lq, Lk, 77)
    if prescaled:
        q = (q.float() * 128 ** -0.5 * LOG2E).to(torch.bfloat16)
        kw, scale = dict(prescaled=True), 1.0 / LOG2E
    else:
        kw, scale = {}, 128 ** -0.5
    whole = N.attn_fwd(q, k, v, n_split=1, **kw)  # a given split: one grid, no tail
    tail = N.attn_fwd(q, k, v, **kw)  # the library's plan: main rounds + tail split
    torch.cuda.synchronize()
    t0 = 12 * 256
    assert torch.equal(tail[:, :, :14], whole[:, :, :14])
    assert torch.equal(tail[:, :t0, 14], whole[:, :t0, 14])
    e_tail = rel_l2(tail[:, t0:, 14:], whole[:, t0:, 14:])
    rows = torch.cat([torch.arange(t0, t0 + 40), torch.arange(Lq - 40, Lq)]).to(device)
    errs = {}
    for h in (14, 15):
        ref = ref_attention(q[:, rows, h:h + 1], k[:, :, h:h + 1], v[:, :, h:h + 1], scale)
        errs[h] = (rel_l2(tail[:, rows, h:h + 1], ref), rel_l2(whole[:, rows, h:h + 1], ref))
    print(f"tail split rows vs the whole launch {e_tail:.2e}; tail / whole vs fp32 {errs}")
    assert 0 < e_tail <= 1.5 * TOL  # two independent bf16 roundings of P (each split has its own shift)
    for h, (et, ew) in errs.items():
        assert et <= TOL and ew <= TOL, errs
