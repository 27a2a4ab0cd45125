"""The reference's attention plug point, served by the MI355X flash kernel.

The reference's `Attention` module calls `self.attn_op(q, k, v)` on [B, S, H, D] tensors and expects
[B, S, H*D] back (minimal_v4_dit.py:377-380, compute_attention :421-432); the op is swapped with
`block.self_attn.register_module("attn_op", op)` (replace_selfattn_op_with_sparse_attn_op :1811) and
wired for context parallelism by `set_context_parallel_group(process_group, ranks, stream)`
(:451-453; MinimalA2AAttnOp a2a_cp.py:208-219). `CP25AttnOp` is that op:

* no CP: q/k/v recast to bf16 (attention() networks/attention.py:107-112, optional q_scale), then
  `cp25_attn_fwd_bounded` (online-max softmax when no norm bounds are given) through libcp25.so;
* CP: q/k/v are this rank's contiguous sequence shard (the reference's split of the sequence); K and
  V of every rank are all-gathered over RCCL in one collective (token-axis all-gather instead of
  the reference's Ulysses all-to-all: same partition, one exchange, no heads % cp constraint) and
  the local queries attend to the full sequence; the output is the local shard.

`attention()` mirrors the reference's functional entry point (networks/attention.py:90-181) for the
options the DiT uses (non-causal, no dropout, no varlen, softmax_scale, q_scale).
"""
from __future__ import annotations

from typing import Any, Optional, Tuple

import torch
import torch.distributed as dist

from . import _native as N

BF16 = torch.bfloat16


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, q_lens=None, k_lens=None, dropout_p: float = 0.0,
              softmax_scale: Optional[float] = None, q_scale: Optional[float] = None, causal: bool = False,
              deterministic: bool = False, dtype: torch.dtype = BF16,
              norm_bounds: Optional[Tuple[float, float]] = None) -> torch.Tensor:
    """networks/attention.py:90-181 on [B, S, H, D] -> [B, S, H, D] (bf16). Options outside the DiT's
    use raise NotImplementedError (the reference raises for unsupported dtypes the same way, :104-105)."""
    if dtype not in (torch.bfloat16, torch.float16, torch.float32):
        raise NotImplementedError(f"{dtype=} is not supported.")
    if dtype != BF16:
        raise NotImplementedError("the MI355X attention kernel computes in bf16 (the reference's DiT dtype)")
    if causal or dropout_p != 0.0 or q_lens is not None or k_lens is not None:
        raise NotImplementedError("causal / dropout / varlen attention is not on the DiT's path")
    del deterministic  # the kernel is deterministic (fixed reduction order)
    q, k, v = q.to(BF16), k.to(BF16), v.to(BF16)
    if q_scale is not None:
        q = q * q_scale
    return N.attn_fwd(q, k, v, softmax_scale=softmax_scale, norm_bounds=norm_bounds)


class CP25AttnOp(torch.nn.Module):
    """Drop-in `Attention.attn_op`: forward(q, k, v [B, S, H, D]) -> [B, S, H*D] bf16."""

    def __init__(self, *args: Any, softmax_scale: Optional[float] = None,
                 norm_bounds: Optional[Tuple[float, float]] = None, **kwargs: Any):
        """norm_bounds: optional (max |q row|, max |k row|) over all rows (e.g. sqrt(D) * max|norm weight|
        after an RMSNorm) enabling the bounded-shift softmax; None = the online-max kernel."""
        del args, kwargs  # MinimalA2AAttnOp(*args, **kwargs) accepts and drops them too
        super().__init__()
        self.softmax_scale = softmax_scale
        self.norm_bounds = norm_bounds
        self.pg = None
        self.stream = None

    def set_context_parallel_group(self, process_group, ranks=None, stream=None) -> None:
        """a2a_cp.py:212-214. The RCCL gather runs on the process group's own stream and is ordered
        against the current stream; `stream` is accepted for signature parity."""
        del ranks
        self.pg = process_group
        self.stream = stream

    def _gather_kv(self, k: torch.Tensor, v: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """All-gather the K/V sequence shards: [B, S, H, D] x 2 -> full-sequence strided views."""
        w = dist.get_world_size(self.pg)
        B, S, H, D = k.shape
        kv = torch.stack([k, v], dim=2).transpose(0, 1).contiguous()  # [S, B, 2, H, D]
        full = torch.empty((w * S, B, 2, H, D), dtype=kv.dtype, device=kv.device)
        if dist.get_backend(self.pg) == "gloo" and kv.is_cuda:
            parts = [torch.empty_like(kv, device="cpu") for _ in range(w)]
            dist.all_gather(parts, kv.cpu(), group=self.pg)
            full.copy_(torch.cat(parts, 0))
        else:
            dist.all_gather_into_tensor(full, kv, group=self.pg)
        return full[:, :, 0].transpose(0, 1), full[:, :, 1].transpose(0, 1)

    def forward(self, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor, *args: Any,
                **kwargs: Any) -> torch.Tensor:
        if args or kwargs.get("video_size") is not None:
            raise NotImplementedError("CP25AttnOp is the dense attention op (no NATTEN video_size)")
        q, k, v = query.to(BF16), key.to(BF16), value.to(BF16)
        if q.dim() != 4 or k.shape != v.shape or k.shape[0] != q.shape[0] or k.shape[2:] != q.shape[2:]:
            raise ValueError(f"expected q/k/v [B, S, H, D], got {tuple(q.shape)} {tuple(k.shape)} {tuple(v.shape)}")
        if self.pg is not None and dist.get_world_size(self.pg) > 1:
            k, v = self._gather_kv(k, v)
        B, S, H, D = q.shape
        o = N.attn_fwd(q, k, v, softmax_scale=self.softmax_scale, norm_bounds=self.norm_bounds)
        return o.reshape(B, S, H * D)
