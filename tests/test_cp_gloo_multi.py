"""CPU, world_size 4 and 8 (gloo): the N > 1 path's host logic at the driver's CP sizes.

* The two-lane pipeline (context_parallel.run_lanes, what dit.forward_tokens drives at CP > 1): each
  lane queues its K/V shard's asynchronous all-gather (a real gloo Work, completed later), yields, and
  waits only on its next step; the event log must show every lane's gather issued before the first
  lane's wait of that block (the overlap), and the sharded attention must equal the unsharded one.
* Token shards whose boundaries fall inside a frame (L = 3 frames x 40 tokens over 4 / 8 ranks; the
  metric's 109 120 tokens over 8 ranks put the 13 640-token boundary inside frame 3): frame indices
  and RoPE rows taken at the shard's global offset, gathered K equal to the full-sequence roped K.
* gather_tokens / split_tokens / broadcast, and the banded VAE decode halo with 4 / 8 bands.
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


T, HP, WP, H, HD = 3, 4, 10, 2, 128
L = T * HP * WP  # 120 tokens; hw = 40


def _full(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(1, L, H, HD, generator=g).to(torch.bfloat16) for _ in range(3)]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cosmos_predict2 import context_parallel as cpx
        from cosmos_predict2.dit import rope_freqs
        from cosmos_predict2.net_config import tiny_dit
        from cosmos_predict2.vae import WanVAE
        from oracle.dit import apply_rope, rope_freqs as orope, sdpa

        grp = dist.group.WORLD
        tok0, n = cpx.token_range(L, grp)
        res = {}
        # ---- RoPE rows at the shard's global token offset (boundaries inside frames)
        cfg = tiny_dit()
        sd = {"pos_embedder.seq": torch.arange(128).float().to(torch.bfloat16),
              "pos_embedder.dim_spatial_range": (torch.arange(0, 42, 2)[:21].float() / 42).to(torch.bfloat16),
              "pos_embedder.dim_temporal_range": (torch.arange(0, 44, 2)[:22].float() / 44).to(torch.bfloat16)}
        import dataclasses

        fr_full = orope(dataclasses.asdict(cfg), T, HP, WP)
        fr_prod = rope_freqs(cfg, T, HP, WP, sd, "cpu")
        res["rope_rows"] = torch.equal(fr_prod[tok0:tok0 + n], fr_full[tok0:tok0 + n])
        frames = torch.arange(tok0, tok0 + n) // (HP * WP)
        res["frame_idx"] = frames[0].item() == tok0 // 40 and frames[-1].item() == (tok0 + n - 1) // 40
        q_full, k_full, v_full = _full(1)
        kr_full = apply_rope(k_full.float(), fr_full).to(torch.bfloat16)
        kr_loc = apply_rope(k_full[:, tok0:tok0 + n].float(), fr_prod[tok0:tok0 + n]).to(torch.bfloat16)
        kr_all = cpx.gather_tokens(kr_loc[0].contiguous(), grp)
        res["roped_k_gather"] = torch.equal(kr_all, kr_full[0])

        # ---- two lanes (CFG cond / uncond), 3 blocks each, async K/V gathers in flight across yields
        log = []
        ref = [sdpa(*_full(10 + b)) for b in range(2)]

        def lane(b):
            qf, kf, vf = _full(10 + b)
            out = None
            for blk in range(3):
                kv = torch.cat([kf[0, tok0:tok0 + n], vf[0, tok0:tok0 + n]], 1).contiguous()  # [n, 2H, hd]
                kv_all = torch.empty((world * n, 2 * H, HD), dtype=kv.dtype)
                work = cpx.all_gather_into_async(kv_all, kv, grp)
                log.append(("issue", blk, b))
                yield blk
                work.wait()
                log.append(("wait", blk, b))
                kk = kv_all[:, :H][None]
                vv = kv_all[:, H:][None]
                out = sdpa(qf[:, tok0:tok0 + n], kk, vv)
            return out

        outs = cpx.run_lanes([lane(0), lane(1)])
        res["lanes_equal_unsharded"] = all(torch.equal(outs[b], ref[b][:, tok0:tok0 + n]) for b in range(2))
        ok_order = True
        for blk in range(3):
            first_wait = log.index(("wait", blk, 0))
            ok_order &= log.index(("issue", blk, 0)) < first_wait and log.index(("issue", blk, 1)) < first_wait
        res["gathers_overlap_other_lane"] = ok_order

        # ---- plumbing helpers
        x = torch.arange(L * 3, dtype=torch.float32).view(L, 3)
        res["split"] = torch.equal(cpx.split_tokens(x, grp), x[tok0:tok0 + n])
        res["gather"] = torch.equal(cpx.gather_tokens(cpx.split_tokens(x, grp), grp), x)
        b = torch.full((2, 3), 7.0) if rank == 0 else torch.empty(0)
        b = cpx.broadcast(b, grp)
        res["broadcast"] = b.shape == (2, 3) and bool(torch.all(b == 7.0))

        # ---- banded VAE decode halo: `world` bands of 2 latent rows each
        R = 2
        full = torch.arange(2 * world * R * 3 * 4, dtype=torch.float32).view(2, world * R, 3, 4)
        vae = WanVAE.__new__(WanVAE)
        vae._band = (grp, rank, world)
        hal = vae._halo(full[:, rank * R:(rank + 1) * R].contiguous())
        padded = torch.cat([torch.zeros(2, 1, 3, 4), full, torch.zeros(2, 1, 3, 4)], 1)
        res["halo"] = torch.equal(hal, padded[:, rank * R:rank * R + R + 2])
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_cp_host_path_world(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, r in res:
        assert all(r.values()), (rank, r)


def test_metric_shard_boundaries_inside_frames():
    """109 120 tokens (31 frames x 44 x 80) over 8 ranks: 13 640 tokens each; every interior boundary
    falls inside a frame, and the per-token frame index of the device kernels (tok // hw) at the
    boundary is the frame the token belongs to."""
    from cosmos_predict2 import context_parallel as cpx

    hw, Lm = 44 * 80, 31 * 44 * 80
    orig = cpx.cp_rank_world
    try:
        for r in range(8):
            cpx.cp_rank_world = lambda group, r=r: (r, 8)
            tok0, n = cpx.token_range(Lm, object())
            assert n == 13640 and tok0 == 13640 * r
            if r:
                assert tok0 % hw != 0  # boundary inside a frame
                assert (tok0 - 1) // hw == tok0 // hw  # the two sides of the boundary share a frame
    finally:
        cpx.cp_rank_world = orig
