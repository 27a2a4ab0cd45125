"""Context-parallel helpers (token sharding over RCCL/xGMI).

The reference splits the latent along T and asserts T % cp == 0
(cosmos_predict2/_src/imaginaire/utils/context_parallel.py:26-54), so T = 31 (121 frames) cannot run
at CP = 2/4/8 there. This build shards the flattened (t, h, w) token axis instead: rank r owns tokens
[r*L/cp, (r+1)*L/cp), every per-token op is local, and self-attention all-gathers K/V
(dit.MinimalV1LVGDiT.forward_tokens). These helpers are the data plumbing around that:
split_inputs_cp / cat_outputs_cp / broadcast equivalents on the token axis.
"""
from __future__ import annotations

from typing import Generator, List, Optional

import torch
import torch.distributed as dist


def cp_rank_world(group) -> tuple[int, int]:
    if group is None:
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def token_range(L: int, group) -> tuple[int, int]:
    """(tok0, n_tok) of this rank; L must divide evenly."""
    r, w = cp_rank_world(group)
    if L % w:
        raise ValueError(f"{L} tokens cannot be split evenly over cp_size {w}")
    n = L // w
    return r * n, n


def split_tokens(x: torch.Tensor, group, dim: int = 0) -> torch.Tensor:
    """Local shard of a replicated token-major tensor (split_inputs_cp on the token axis)."""
    tok0, n = token_range(x.shape[dim], group)
    return x.narrow(dim, tok0, n).contiguous()


def all_gather_into(out: torch.Tensor, x: torch.Tensor, group) -> torch.Tensor:
    """out[r*n:(r+1)*n] = rank r's x. RCCL (`nccl` backend) gathers straight between HBM buffers;
    the gloo backend (CPU tests, or several ranks sharing one GPU in tests) stages through host memory."""
    if dist.get_backend(group) == "gloo" and x.is_cuda:
        w = dist.get_world_size(group)
        xc = x.detach().contiguous().cpu()
        parts = [torch.empty_like(xc) for _ in range(w)]
        dist.all_gather(parts, xc, group=group)
        out.view((w * xc.shape[0],) + tuple(xc.shape[1:])).copy_(torch.cat(parts, 0))
        return out
    w = dist.get_world_size(group)
    # the concatenated [w * x0, ...] form (every backend accepts it; out may be given stacked)
    dist.all_gather_into_tensor(out.view((w * x.shape[0],) + tuple(x.shape[1:])), x.contiguous(), group=group)
    return out


class _Done:
    """Handle of a collective that already completed (tools that substitute local copies for the gather)."""

    def wait(self) -> bool:
        return True


class _GlooDeferred:
    """Handle of a gloo all-gather of device data still in flight (tests; several ranks sharing one GPU): the
    shard was staged to host memory at issue, the gloo collective runs asynchronously, and wait() lands the
    gathered bytes in `out` on the CURRENT stream, so `out` is written only after wait() -- the ordering RCCL's
    async work gives the lanes of run_lanes (the other lane's block is queued between issue and wait)."""

    def __init__(self, out: torch.Tensor, src: torch.Tensor, parts, work, w: int, row_shape):
        # src (the staged shard) and parts stay referenced until wait(): the async gloo work reads / writes them
        self.out, self.src, self.parts, self.work, self.w, self.row_shape = out, src, parts, work, w, row_shape

    def wait(self) -> bool:
        self.work.wait()
        self.out.view((self.w * self.parts[0].shape[0],) + self.row_shape).copy_(torch.cat(self.parts, 0))
        return True


def all_gather_into_async(out: torch.Tensor, x: torch.Tensor, group):
    """Asynchronous all_gather_into: returns a handle whose .wait() makes the CURRENT stream wait for
    the gather. With RCCL the gather runs on the process group's own stream, ordered after the work
    already queued on the current stream (so x is complete), and overlaps whatever the current
    stream does next; the gloo path (tests) stages x to the host and completes the gather in wait()."""
    if dist.get_backend(group) == "gloo" and x.is_cuda:
        w = dist.get_world_size(group)
        xc = x.detach().contiguous().cpu()
        parts = [torch.empty_like(xc) for _ in range(w)]
        work = dist.all_gather(parts, xc, group=group, async_op=True)
        return _GlooDeferred(out, xc, parts, work, w, tuple(xc.shape[1:]))
    w = dist.get_world_size(group)
    return dist.all_gather_into_tensor(out.view((w * x.shape[0],) + tuple(x.shape[1:])), x.contiguous(),
                                       group=group, async_op=True)


def run_lanes(lanes: List[Generator]) -> list:
    """Round-robin driver of software-pipelined lanes on ONE stream (dit.forward_tokens, CP > 1).

    Each lane is a generator that queues device work on the current stream, starts an asynchronous
    collective (all_gather_into_async), yields, and on its next step waits for that collective
    (`work.wait()`: the current stream waits for the collective's completion event) before queueing
    the work that reads the gathered data. Driving the lanes in rotation queues lane b+1's whole
    block between lane b's gather and lane b's wait, so the transfer overlaps that compute.

    Stream / allocator invariant this relies on (and why the lanes are not on separate streams):
      * every kernel and every work.wait() is on the one current stream, so program order is
        stream order: no event edges between compute streams exist to mis-order or deadlock;
      * every tensor is allocated and freed on that stream (caching-allocator pool of the current
        stream); the only buffers another stream touches are a collective's input and output, which
        the process group keeps alive (record_stream / stash) until the collective's stream is done;
      * a round-1 variant ran the lanes on two streams with cross-stream events (lane 1 waiting on
        an event lane 0 recorded after queueing its gather) and hung intermittently in device
        synchronisation when two ranks shared one GPU over gloo. The hazard that variant had and
        this one cannot: HIP multiplexes streams onto a few hardware queues per process
        (GPU_MAX_HW_QUEUES = 4 here; default + 2 lanes + the gloo staging copies + RCCL's stream
        already exceed it), and an event-wait packet at the head of a shared hardware queue blocks
        every stream mapped behind it; with the gloo staging path doing blocking host copies inside
        a lane, a wait queued ahead of the record it depends on (in another stream sharing the
        queue) cannot drain. One stream has no such edge.
    Returns each lane's return value, in lane order."""
    live = [True] * len(lanes)
    out = [None] * len(lanes)
    while any(live):
        for i, g in enumerate(lanes):
            if not live[i]:
                continue
            try:
                next(g)
            except StopIteration as e:
                out[i] = e.value
                live[i] = False
    return out


def kv_chunk_views(kv_all_c: torch.Tensor, n_tok_total: int, B: int, Hc: int, hd: int):
    """K and V [B, L, Hc, hd] views of one gathered head chunk [L*B, 2*Hc*hd] (rows token-major,
    batch inner; each row = Hc K heads then Hc V heads), as the attention kernel reads them."""
    kc = kv_all_c.view(n_tok_total, B, 2, Hc, hd)
    return kc[:, :, 0].transpose(0, 1), kc[:, :, 1].transpose(0, 1)


def gather_tokens(x: torch.Tensor, group) -> torch.Tensor:
    """Concatenate every rank's token shard along dim 0 (cat_outputs_cp on the token axis)."""
    r, w = cp_rank_world(group)
    if w == 1:
        return x
    out = torch.empty((w * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    return all_gather_into(out, x, group)


def broadcast(x: Optional[torch.Tensor], group, src_in_group: int = 0) -> Optional[torch.Tensor]:
    """Broadcast from the group's first rank (robust_broadcast: shape first, then data)."""
    r, w = cp_rank_world(group)
    if w == 1 or x is None:
        return x
    src = dist.get_global_rank(group, src_in_group)
    dev = x.device
    shape = torch.tensor(list(x.shape), dtype=torch.int64, device=dev)
    n = torch.tensor([shape.numel()], dtype=torch.int64, device=dev)
    dist.broadcast(n, src, group=group)
    if r != src_in_group:
        shape = torch.empty(int(n.item()), dtype=torch.int64, device=dev)
    dist.broadcast(shape, src, group=group)
    if r != src_in_group:
        x = torch.empty(shape.tolist(), dtype=x.dtype, device=dev)
    x = x.contiguous()
    dist.broadcast(x, src, group=group)
    return x
