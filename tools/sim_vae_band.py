"""Compute time of one context-parallel rank's banded VAE decode, simulated on one GPU.

Rank 0 of N decodes its h/N latent rows of the metric's latent [1, 16, 31, 88, 160] (121 frames at
704x1280) exactly as on a real rank, except that the RCCL all-gathers (halo rows, middle-attention
K/V, final bands) are local copies (this rank's data repeated N times: same bytes, no xGMI traffic).
Prints one JSON line per N with the decode seconds (compare with the N = 1 decode / N).
usage: python tools/sim_vae_band.py [--cp 1 2 4 8] [--frames 31]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import context_parallel as cpx  # noqa: E402
from cosmos_predict2.vae import Wan2pt1VAEInterface, init_vae_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cp", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--frames", type=int, default=31)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tok = Wan2pt1VAEInterface(init_vae_state_dict(seed=1, device=dev), device=dev)
    z = torch.randn(1, 16, a.frames, 88, 160, device=dev)
    state = {"n": 1}

    def fake_gather(out, x, group):
        n = state["n"]
        for r in range(n):
            out.view((n,) + tuple(x.shape))[r].copy_(x)
        return out

    cpx.all_gather_into = fake_gather
    cpx.cp_rank_world = lambda group: (0, state["n"]) if group is not None else (0, 1)
    for n in a.cp:
        state["n"] = n
        tok.set_context_parallel_group(None if n == 1 else object())
        tok.decode(z[:, :, :2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        v = tok.decode(z)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"cp": n, "latent_frames": a.frames, "decode_s": dt, "out": list(v.shape)}), flush=True)


if __name__ == "__main__":
    main()
