"""The reference's operator plug point: `Attention.attn_op` swapped for CP25AttnOp.

A minimal module shaped like the reference's `Attention` (minimal_v4_dit.py:321-453: q/k/v/output
projections, per-head RMSNorm of q and k, `self.attn_op(q, k, v)` -> [B, S, H*D], output_proj) gets
its op replaced the way replace_selfattn_op_with_sparse_attn_op does it (`register_module("attn_op",
op)`, :1811); its forward must match the oracle's SDPA restatement (networks/attention.py:90-181).
CP: two ranks (gloo, sharing cuda:0) call the op on their sequence shards after
`set_context_parallel_group(pg, ranks, stream)` (a2a_cp.py:212-214); the shards of the output must
equal the single-rank output bit for bit (no key-range split: same keys, same order).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import __graft_entry__  # noqa: F401
from cosmos_predict2 import _native as N  # noqa: E402

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16


class _Attention(torch.nn.Module):
    """Reference-shaped Attention (minimal_v4_dit.py:321-453) with a placeholder attn_op."""

    def __init__(self, dim: int, heads: int, context_dim=None):
        super().__init__()
        self.n_heads, self.head_dim = heads, dim // heads
        cd = dim if context_dim is None else context_dim
        self.q_proj = torch.nn.Linear(dim, dim, bias=False)
        self.k_proj = torch.nn.Linear(cd, dim, bias=False)
        self.v_proj = torch.nn.Linear(cd, dim, bias=False)
        self.output_proj = torch.nn.Linear(dim, dim, bias=False)
        self.q_w = torch.nn.Parameter(torch.ones(self.head_dim))
        self.k_w = torch.nn.Parameter(torch.ones(self.head_dim))
        self.attn_op = torch.nn.Identity()  # the reference builds its own op here; swapped below

    def _rms(self, x, w):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * w.float()).to(x.dtype)

    def compute_qkv(self, x, context=None):
        context = x if context is None else context
        B = x.shape[0]
        q = self.q_proj(x).view(B, -1, self.n_heads, self.head_dim)
        k = self.k_proj(context).view(B, -1, self.n_heads, self.head_dim)
        v = self.v_proj(context).view(B, -1, self.n_heads, self.head_dim)
        return self._rms(q, self.q_w), self._rms(k, self.k_w), v

    def forward(self, x, context=None):
        q, k, v = self.compute_qkv(x, context)
        return self.output_proj(self.attn_op(q, k, v))


def _module(dev, dim=512, heads=4, context_dim=None, seed=0):
    torch.manual_seed(seed)
    m = _Attention(dim, heads, context_dim).to(dev, BF16)
    with torch.no_grad():
        m.q_w.uniform_(0.5, 1.5)
        m.k_w.uniform_(0.5, 1.5)
    return m


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("B,S,Sc", [(1, 333, None), (2, 1000, None), (2, 777, 512)])
def test_attn_op_registered_matches_oracle(device, B, S, Sc):
    from cosmos_predict2.attn_op import CP25AttnOp
    from oracle.dit import sdpa

    m = _module(device, context_dim=256 if Sc else None)
    m.register_module("attn_op", CP25AttnOp())
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, S, 512, generator=g).to(device, BF16)
    ctx = torch.randn(B, Sc, 256, generator=g).to(device, BF16) if Sc else None
    with torch.no_grad():
        out = m(x, ctx)
        q, k, v = m.compute_qkv(x, ctx)
        ref = m.output_proj(sdpa(q.cpu(), k.cpu(), v.cpu()).to(device))
        core = m.attn_op(q, k, v)
    assert out.shape == (B, S, 512) and core.shape == (B, S, 512)
    e_core = _rel(core.cpu(), sdpa(q.cpu(), k.cpu(), v.cpu()))
    e = _rel(out, ref)
    print(f"attn_op core rel-L2 {e_core:.2e}, module {e:.2e}")
    assert e_core <= 4e-3 and e <= 6e-3  # P and O rounded to bf16 in the kernel (~2e-3 floor)


def test_attention_function_options(device):
    from cosmos_predict2.attn_op import attention
    from oracle.dit import sdpa

    g = torch.Generator().manual_seed(2)
    q, k, v = (torch.randn(1, 200, 2, 128, generator=g) for _ in range(3))
    out = attention(q.to(device), k.to(device), v.to(device), q_scale=0.5)  # fp32 in -> recast to bf16
    ref = sdpa((q.to(BF16) * 0.5), k.to(BF16), v.to(BF16)).view(1, 200, 2, 128)
    assert _rel(out.cpu(), ref) <= 4e-3
    with pytest.raises(NotImplementedError):
        attention(q.to(device), k.to(device), v.to(device), causal=True)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    g = torch.Generator().manual_seed(5)
    B, S, H = 2, 640, 4
    return [torch.randn(B, S, H, 128, generator=g).to(BF16) for _ in range(3)]


def _worker(rank, world, port, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    N.set_attn_split(1)  # no key split: rows equal to the single-rank run bit for bit
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cosmos_predict2.attn_op import CP25AttnOp

        dev = torch.device("cuda:0")
        q, k, v = _case()
        n = q.shape[1] // world
        sl = slice(rank * n, (rank + 1) * n)
        op = CP25AttnOp()
        op.set_context_parallel_group(dist.group.WORLD, list(range(world)), torch.cuda.Stream(dev))
        out = op(q[:, sl].to(dev), k[:, sl].to(dev), v[:, sl].to(dev))
        torch.cuda.synchronize(dev)
        q_out.put((rank, out.cpu().float().numpy()))
    finally:
        dist.destroy_process_group()


def test_attn_op_context_parallel_matches_single_rank(device, monkeypatch):
    from cosmos_predict2.attn_op import CP25AttnOp

    monkeypatch.setattr(N, "_ATTN_SPLIT", 1)
    q, k, v = _case()
    ref = CP25AttnOp()(q.to(device), k.to(device), v.to(device)).cpu().float()
    ctx = mp.get_context("spawn")
    qo = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, qo)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(qo.get(timeout=100) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in ps)
    got = torch.cat([torch.from_numpy(res[0]), torch.from_numpy(res[1])], 1)
    assert torch.equal(got, ref)
