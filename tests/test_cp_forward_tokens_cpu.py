"""CPU, gloo, world 2 and 4: the real dit.MinimalV1LVGDiT.forward_tokens on a token shard, its two CFG lanes driven by
context_parallel.run_lanes with asynchronous all-gathers (a real gloo Work, completed only when the lane waits),
against the CP = 1 forward of the whole sequence.

The libcp25 kernels are replaced by the CPU stand-ins of tests/cpu_kernels.py (the reference's op sequences in torch
CPU ops), so what runs here is exactly the product's host path: token sharding with boundaries inside frames, the
per-lane block loop (dit._blocks), the K|V export (copy_rows), the asynchronous gather and the yield before its
wait (dit._cp_self_attention), RoPE rows at the shard's global offset, the per-frame modulation rows, the final
layer. Checks: every rank's output rows equal the same rows of the CP = 1 forward (rel-L2 <= 5e-3, measured 6-9e-4: the CPU bf16
GEMMs of M rows vs all rows may round differently; the GPU tests hold the device path to bit-exactness), and the
event log shows each lane's gather of block k issued before the other lane's wait of block k (the overlap)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import __graft_entry__  # noqa: F401  (import paths)

T, HP, WP = 3, 4, 8  # 96 tokens, hw 32: shard boundaries at 48 / 24, 72 fall inside frames for world 4


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
        from cosmos_predict2 import context_parallel as cpx
        from cosmos_predict2 import dit as dit_mod
        from cosmos_predict2.dit import Geometry, MinimalV1LVGDiT, init_state_dict
        from cosmos_predict2.net_config import tiny_dit

        res = {}
        with cpu_kernels.patched(), torch.no_grad():
            cfg = tiny_dit(num_blocks=2)
            sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=3, zero_adaln_out=False).items()}
            net = MinimalV1LVGDiT(cfg, device="cpu")
            net.load_state_dict(sd)
            L = T * HP * WP
            g = torch.Generator().manual_seed(7)
            rows = torch.randn(L, 2, 72, generator=g).to(torch.bfloat16)
            t_B_T = torch.tensor([[0.0001, 0.5, 0.5], [0.0001, 0.5, 0.5]])
            ctx = net.prepare_context(torch.randn(2, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16))
            ref = net.forward_tokens(rows, t_B_T, ctx, Geometry(T=T, Hp=HP, Wp=WP, tok0=0, n_tok=L))

            log = []
            orig = dit_mod.all_gather_into_async

            class Logged:
                def __init__(self, work, j):
                    self.work, self.j = work, j

                def wait(self):
                    log.append(("wait", self.j))
                    return self.work.wait()

            def gather(out, x, group):
                work = orig(out, x, group)
                j = sum(1 for e in log if e[0] == "issue")
                log.append(("issue", j))
                res.setdefault("deferred", work is not None and not isinstance(work, cpx._Done))
                return Logged(work, j)

            dit_mod.all_gather_into_async = gather
            try:
                grp = dist.group.WORLD
                net.cp_group = grp
                tok0, n = cpx.token_range(L, grp)
                out = net.forward_tokens(rows[tok0:tok0 + n], t_B_T, ctx, Geometry(T=T, Hp=HP, Wp=WP, tok0=tok0, n_tok=n))
            finally:
                dit_mod.all_gather_into_async = orig
                net.cp_group = None
            exp = ref[tok0:tok0 + n]
            res["rel"] = ((out - exp).float().norm() / exp.float().norm()).item()
            res["shape"] = tuple(out.shape) == tuple(exp.shape)
            issues = [e for e in log if e[0] == "issue"]
            res["gathers"] = len(issues)
            pos = {e: i for i, e in enumerate(log)}
            # issue 2k + 1 (lane 1, block k) before wait 2k (lane 0, block k)
            res["overlap"] = all(pos[("issue", 2 * k + 1)] < pos[("wait", 2 * k)] for k in range(len(issues) // 2))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_forward_tokens_cp_lanes_gloo(world):
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
    for rank, r in res:
        print(f"world {world} rank {rank}: {r}")
        assert r["shape"] and r["deferred"] and r["overlap"], (rank, r)
        assert r["gathers"] == 2 * 2, (rank, r)  # 2 blocks x 2 lanes
        assert r["rel"] <= 5e-3, (rank, r)
