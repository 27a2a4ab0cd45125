"""CPU, world_size 2 (gloo): the context-parallel token sharding of the N > 1 path.

The device path shards the flattened (t, h, w) token axis over ranks and all-gathers K/V inside
self-attention (dit.MinimalV1LVGDiT.forward_tokens); everything else is per token. Here the same
decomposition runs on the CPU with gloo on the oracle's attention and checks it equals the
unsharded computation; plus the gather / split / broadcast helpers used around the sampler.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import __graft_entry__  # noqa: F401


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cosmos_predict2 import context_parallel as cpu
        from oracle.dit import sdpa

        g = torch.Generator().manual_seed(0)
        L, B, H, hd = 96, 2, 2, 128
        q_full = torch.randn(B, L, H, hd, generator=g).to(torch.bfloat16)
        k_full = torch.randn(B, L, H, hd, generator=g).to(torch.bfloat16)
        v_full = torch.randn(B, L, H, hd, generator=g).to(torch.bfloat16)
        ref = sdpa(q_full, k_full, v_full)
        tok0, n = cpu.token_range(L, dist.group.WORLD)
        # local shards in the device layout [tokens, B, ...]
        kv_loc = torch.cat([k_full, v_full], 2)[:, tok0:tok0 + n].transpose(0, 1).contiguous()  # [n, B, 2H, hd]
        kv = cpu.gather_tokens(kv_loc, dist.group.WORLD)  # [L, B, 2H, hd]
        k = kv[:, :, :H].transpose(0, 1)
        v = kv[:, :, H:].transpose(0, 1)
        out_loc = sdpa(q_full[:, tok0:tok0 + n], k, v)
        ok_attn = torch.equal(out_loc, ref[:, tok0:tok0 + n])
        # the device path's pipelined form: K/V packed per head chunk [n*B, 2*Hc*hd], each chunk
        # all-gathered asynchronously, attention per chunk on the gathered views
        nc = 2
        Hc = H // nc
        kl = k_full[:, tok0:tok0 + n].transpose(0, 1)  # [n, B, H, hd]
        vl = v_full[:, tok0:tok0 + n].transpose(0, 1)
        works, alls = [], []
        for c in range(nc):
            loc = torch.cat([kl[:, :, c * Hc:(c + 1) * Hc], vl[:, :, c * Hc:(c + 1) * Hc]], 2).reshape(n * B, -1)
            alls.append(torch.empty((2 * n * B, loc.shape[1]), dtype=loc.dtype))
            works.append(cpu.all_gather_into_async(alls[c], loc, dist.group.WORLD))
        ok_chunks = True
        for c in range(nc):
            works[c].wait()
            kc, vc = cpu.kv_chunk_views(alls[c], L, B, Hc, hd)
            oc = sdpa(q_full[:, tok0:tok0 + n, c * Hc:(c + 1) * Hc], kc, vc)
            ok_chunks &= torch.equal(oc.view(B, n, Hc, hd), ref.view(B, L, H, hd)[:, tok0:tok0 + n, c * Hc:(c + 1) * Hc])
        ok_attn = ok_attn and ok_chunks
        # sampler plumbing helpers
        x = torch.arange(L * 3, dtype=torch.float32).view(L, 3)
        ok_split = torch.equal(cpu.split_tokens(x, dist.group.WORLD), x[tok0:tok0 + n])
        ok_gather = torch.equal(cpu.gather_tokens(cpu.split_tokens(x, dist.group.WORLD), dist.group.WORLD), x)
        b = torch.full((2, 3), float(rank)) if rank == 0 else torch.empty(0)
        b = cpu.broadcast(b, dist.group.WORLD)
        ok_bcast = b.shape == (2, 3) and torch.all(b == 0).item()
        # VAE decode bands: the halo rows of a band are its neighbours' edge rows, zeros at the edges
        from cosmos_predict2.vae import WanVAE

        full = torch.arange(2 * 8 * 3 * 4, dtype=torch.float32).view(2, 8, 3, 4)  # [T, h, w, C]
        vae = WanVAE.__new__(WanVAE)
        vae._band = (dist.group.WORLD, rank, 2)
        band = full[:, rank * 4:(rank + 1) * 4].contiguous()
        hal = vae._halo(band)
        padded = torch.cat([torch.zeros(2, 1, 3, 4), full, torch.zeros(2, 1, 3, 4)], 1)
        ok_halo = torch.equal(hal, padded[:, rank * 4:rank * 4 + 6])
        q.put((rank, ok_attn, ok_split, ok_gather, ok_bcast, ok_halo))
    finally:
        dist.destroy_process_group()


def test_cp_token_sharding_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in res:
        assert all(r[1:]), r


def test_token_range_rejects_uneven():
    from cosmos_predict2 import context_parallel as cpu

    def world(r, w):  # cp_rank_world stand-in: the divisibility check needs only (rank, world)
        return lambda group: (r, w)

    orig = cpu.cp_rank_world
    try:
        cpu.cp_rank_world = world(1, 3)
        with pytest.raises(ValueError):
            cpu.token_range(109120, object())  # 720p x 121f: 109120 tokens, not divisible by 3
        for w in (1, 2, 4, 8):  # the CP sizes the bench runs all divide 109120
            cpu.cp_rank_world = world(w - 1, w)
            assert cpu.token_range(109120, object()) == ((w - 1) * (109120 // w), 109120 // w)
    finally:
        cpu.cp_rank_world = orig
