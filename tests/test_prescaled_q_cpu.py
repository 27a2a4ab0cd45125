"""Why the DiT's prescaled query costs no parity (VERDICT r3 "weak" 1 / next 7), on the CPU in fp32 arithmetic.

The reference rounds the normed, roped q to bf16 and applies softmax_scale to the fp32 scores
(minimal_v4_dit.py:411-419; networks/attention.py:107-112). The DiT here emits bf16(q * c), c = scale * log2(e), from the
RMSNorm/RoPE kernel's fp32 result (cp25_head_rmsnorm_rope out_scale) and runs exp2 on the scores. Both round the query
ONCE at the same relative precision, so against attention on the unrounded fp32 q they sit at the same distance. The
21 % gap round 3's op table showed (2.80e-3 vs 2.31e-3) came from the test rounding twice, bf16(bf16(q) * c): the
prescaled kernel was fed an already rounded q. Measured here with P kept in fp32 (the q effect alone) and with P
rounded to bf16 before P.V (what the kernels do)."""
import math

import pytest
import torch

BF16 = torch.bfloat16


def _att(q, k, v, scale, p_bf16):
    s = torch.einsum("blhd,bmhd->bhlm", q, k) * scale
    if not p_bf16:
        return torch.einsum("bhlm,bmhd->blhd", torch.softmax(s, -1), v)
    e = torch.exp(s - s.amax(-1, keepdim=True)).to(BF16).float()
    return torch.einsum("bhlm,bmhd->blhd", e, v) / e.sum(-1).transpose(1, 2)[..., None]


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("p_bf16", [False, True])
def test_one_rounding_of_q_times_c_equals_one_rounding_of_q(p_bf16):
    g = torch.Generator().manual_seed(0)
    B, L, Lk, H = 1, 512, 2048, 2
    q = torch.randn(B, L, H, 128, generator=g)
    q = q * torch.rsqrt(q.pow(2).mean(-1, keepdim=True))
    k = torch.randn(B, Lk, H, 128, generator=g)
    k = (k * torch.rsqrt(k.pow(2).mean(-1, keepdim=True))).to(BF16).float()
    v = torch.randn(B, Lk, H, 128, generator=g).to(BF16).float()
    scale = 128 ** -0.5
    c = scale * math.log2(math.e)
    truth = _att(q, k, v, scale, False)
    ref = _rel(_att(q.to(BF16).float(), k, v, scale, p_bf16), truth)                      # reference rounding point
    dit = _rel(_att((q * c).to(BF16).float(), k, v, 1 / math.log2(math.e), p_bf16), truth)  # DiT: q * c rounded once
    dbl = _rel(_att((q.to(BF16).float() * c).to(BF16).float(), k, v, 1 / math.log2(math.e), p_bf16), truth)
    print(f"P {'bf16' if p_bf16 else 'fp32'}: reference {ref:.3e}, DiT prescaled {dit:.3e}, double-rounded {dbl:.3e}")
    assert abs(dit - ref) <= 0.03 * ref
    assert dbl >= 1.15 * ref  # the artifact the round-3 op table measured
