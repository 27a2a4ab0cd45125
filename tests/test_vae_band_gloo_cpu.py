"""The context-parallel VAE decode's band plumbing at world 2 and 4 over real gloo collectives, on the CPU.

Reference: the spatial context parallelism of the Wan2.1 tokenizer plugins (cosmos_predict2/_src/predict2/tokenizers/
wan2pt1_2d_plugins.py:139-310): each rank decodes a band of latent rows. Here (vae.WanVAE.decode) rank r decodes
latent rows [r h/N, (r+1) h/N) of every frame: every 3x3 conv gets its neighbours' edge rows through an all-gather
(_halo; zero rows at the image edge), the nearest-2x upsample conv reads the haloed low-res band with pads -1, the
middle AttentionBlock all-gathers K/V of the whole frame, and the bands are all-gathered at the end. The libcp25
kernels are replaced by test-only torch stand-ins (tests/cpu_kernels.py: float64 arithmetic rounded once to bf16, so a
pixel's value does not depend on the extent of the call that computed it); the band logic, the halo exchange and the
collectives are the product's own. Every rank must end with the unbanded decode, bit for bit."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import __graft_entry__  # noqa: F401  (sys.path)
import cpu_kernels
from cosmos_predict2.vae import WanVAE, init_vae_state_dict


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    torch.manual_seed(0)
    sd = init_vae_state_dict(seed=2)
    z = torch.randn(1, 16, 2, 8, 6, generator=torch.Generator().manual_seed(5))
    return sd, z


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with cpu_kernels.patched():
            sd, z = _case()
            vae = WanVAE(sd, device="cpu")
            vae.cp_group = dist.group.WORLD
            out = vae.decode(z)
        q.put((rank, out.float().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_banded_decode_matches_full(world):
    torch.set_num_threads(4)
    with cpu_kernels.patched():
        sd, z = _case()
        full = WanVAE(sd, device="cpu").decode(z).float()
    assert full.shape == (1, 3, 5, 64, 48)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {r: torch.from_numpy(a) for r, a in (q.get(timeout=600) for _ in ps)}
    for p in ps:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in ps)
    for r in range(world):
        assert torch.equal(res[r], full), (r, (res[r] - full).abs().max().item())
