"""The oracle's flash-attention SDPA mode (oracle.dit.flash_sdpa, bf16 P for P.V as the flash / cuDNN kernels the
reference dispatches to, networks/attention.py:119-178) against a step-by-step restatement of FlashAttention-2's
forward (Algorithm 1: key blocks in order, running max, rescaled O and row sum over the unrounded fp32 P). The oracle
vectorises the running max; both must agree to fp32 reordering (a few bf16 output flips), and the bf16-P form must sit
at the bf16 floor from the fp32 truth (parity unpinned: no fixture of those kernels exists here)."""
import math

import torch

from oracle import dit as odit


def _flash_sequential(q, k, v, blk=128):
    B, L, H, D = q.shape
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    c = D ** -0.5 * math.log2(math.e)
    m = torch.full(qf.shape[:-1], -float("inf"))
    l = torch.zeros(qf.shape[:-1])
    o = torch.zeros(qf.shape)
    for j in range(0, kf.shape[2], blk):
        s = qf @ kf[:, :, j:j + blk].transpose(-1, -2)
        mn = torch.maximum(m, s.amax(-1))
        r = torch.exp2((m - mn) * c)
        p = torch.exp2(s * c - mn[..., None] * c)
        l = l * r + p.sum(-1)
        o = o * r[..., None] + p.to(torch.bfloat16).float() @ vf[:, :, j:j + blk]
        m = mn
    return (o / l[..., None]).transpose(1, 2).reshape(B, L, H * D).to(torch.bfloat16)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_flash_sdpa_matches_sequential_flash():
    g = torch.Generator().manual_seed(0)
    B, L, Lk, H = 1, 300, 1000, 2  # ragged last key block
    q, k, v = (torch.randn(B, n, H, 128, generator=g) for n in (L, Lk, Lk))
    q = (q * torch.rsqrt(q.pow(2).mean(-1, keepdim=True))).to(torch.bfloat16)
    k = (k * torch.rsqrt(k.pow(2).mean(-1, keepdim=True)) * 3).to(torch.bfloat16)  # trained-size scores
    v = v.to(torch.bfloat16)
    s = torch.einsum("blhd,bmhd->bhlm", q.float(), k.float()) * 128 ** -0.5
    truth = torch.einsum("bhlm,bmhd->blhd", torch.softmax(s, -1), v.float()).reshape(B, L, H * 128)
    fp32p = odit.sdpa(q, k, v)
    with odit.flash_sdpa():
        flash = odit.sdpa(q, k, v)
    assert odit._SDPA == ["fp32p"]
    assert rel(flash, _flash_sequential(q, k, v)) < 1e-4
    # both at the bf16 floor from the truth; the bf16 P costs a little more than the fp32 P
    assert rel(fp32p, truth) < 3e-3 and rel(flash, truth) < 3e-3
    assert rel(flash, truth) >= rel(fp32p, truth) * 0.95
