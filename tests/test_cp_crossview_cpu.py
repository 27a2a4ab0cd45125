"""CPU, gloo, world 2: the cross-view net (MultiViewCrossDiT, predict2_multiview/networks/multiview_cross_dit.py) under
context parallelism. Each rank holds frames [rank Tl, (rank + 1) Tl) of every view
(Geometry.frame_shard, the reference's "B C (c V T) H W" CP layout, multiview_vid2vid_model_rectified_flow.py:400-403),
so the cross-view attention of a frame is local (CrossViewAttention needs no communication, multiview_cross_dit.py:
230-231) and each view's self-attention gathers the other ranks' frames of that view (dit._cp_self_attention with
views). The real dit.MinimalV1LVGDiT.forward_tokens runs its two CFG lanes over real asynchronous gloo all-gathers,
with the libcp25 kernels replaced by tests/cpu_kernels.py; every rank's rows must equal the same global rows of the
CP = 1 forward (rel-L2 <= 5e-3: CPU bf16 GEMMs over fewer rows may round differently, as in
test_cp_forward_tokens_cpu.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import __graft_entry__  # noqa: F401  (import paths)

V, TV, HP, WP = 3, 4, 4, 8  # 3 views x 4 frames x 32 tokens
MAP = ((1, 2), (0,), (0, 1))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cpu_kernels
        from cosmos_predict2 import dit as dit_mod
        from cosmos_predict2.dit import Geometry, MinimalV1LVGDiT, init_state_dict
        from cosmos_predict2.net_config import tiny_dit

        res = {}
        with cpu_kernels.patched(), torch.no_grad():
            cfg = tiny_dit(num_blocks=2, n_cameras_emb=3, state_t=TV, adaln_view_embedding=True,
                           cross_view_attn_map=MAP, use_wan_fp32_strategy=False)
            sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=3, zero_adaln_out=False).items()}
            net = MinimalV1LVGDiT(cfg, device="cpu")
            net.load_state_dict(sd)
            T = V * TV
            L = T * HP * WP
            g = torch.Generator().manual_seed(7)
            rows = torch.randn(L, 1, 72, generator=g).to(torch.bfloat16)
            t_B_T = torch.linspace(0.1, 0.9, T)[None].expand(2, T).contiguous()
            ctx = net.prepare_context(torch.randn(2, 512 * V, cfg.crossattn_proj_in_channels,
                                                  generator=g).to(torch.bfloat16))
            vi = torch.tensor([2, 0, 1])  # view ids in input order (a permuted rig)
            ref = net.forward_tokens(rows, t_B_T, ctx, Geometry(T=T, Hp=HP, Wp=WP, tok0=0, n_tok=L, n_views=V),
                                     view_indices=vi)
            orig = dit_mod.all_gather_into_async
            n_gather = []

            def gather(out_, x, group):
                n_gather.append(x.shape)
                return orig(out_, x, group)

            dit_mod.all_gather_into_async = gather
            net.cp_group = dist.group.WORLD
            try:
                geo = Geometry.frame_shard(T, HP, WP, V, rank, world)
                ids = geo.token_ids()
                out = net.forward_tokens(rows[ids].contiguous(), t_B_T, ctx, geo, view_indices=vi)
            finally:
                net.cp_group = None
                dit_mod.all_gather_into_async = orig
            res["gathers"] = len(n_gather)
            exp = ref[ids]
            res["rel"] = ((out - exp).float().norm() / exp.float().norm()).item()
            res["shape"] = tuple(out.shape) == tuple(exp.shape)
            res["frames"] = geo.frames
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_crossview_cp_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, r in sorted(res):
        print(f"cross-view CP world {world} rank {rank}: {r}")
        assert r["shape"] and r["gathers"] == 2 * 2, (rank, r)  # 2 blocks x 2 CFG lanes
        assert r["rel"] <= 5e-3, (rank, r)
    assert sorted(res)[0][1]["frames"] == (0, 1, 4, 5, 8, 9)


def test_frame_shard_geometry():
    from cosmos_predict2.dit import Geometry

    g = Geometry.frame_shard(12, 2, 3, 3, 1, 2)  # 3 views x 4 frames, rank 1 of 2: frames 2, 3 of each view
    assert g.frames == (2, 3, 6, 7, 10, 11) and g.n_tok == 36
    ids = g.token_ids()
    assert ids[:7].tolist() == [12, 13, 14, 15, 16, 17, 18] and ids[-1].item() == 71
    lg = g.local()
    assert (lg.T, lg.T_view, lg.n_views, lg.tok0, lg.n_tok, lg.frames) == (6, 2, 3, 0, 36, None)
    allids = torch.cat([Geometry.frame_shard(12, 2, 3, 3, r, 2).token_ids() for r in range(2)])
    assert torch.equal(allids.sort().values, torch.arange(72))
    with pytest.raises(ValueError):
        Geometry.frame_shard(12, 2, 3, 3, 0, 3)  # 4 frames per view over 3 ranks
