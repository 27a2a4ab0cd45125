"""Correctness sweep of one build of cp25_attn_fwd (lab or in-tree) against fp32 math.

usage: python tools/check_attn_lib.py [--lib tools/lab/libcp25_x.so]
Shapes cover ragged key tiles, Lk < one tile, partial query blocks and key-range splits; prints one
JSON line per shape and exits non-zero if any rel-L2 exceeds 4e-3.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    if a.lib:
        N._LIB_PATH = a.lib
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    bad = 0
    for (B, H, Lq, Lk, ns, scale) in [(1, 2, 300, 1, 1, 1.0), (1, 2, 256, 64, 1, 1.0), (1, 1, 100, 65, 1, 1.0),
                                     (2, 3, 513, 200, 1, 1.0), (1, 2, 1000, 1000, 1, 1.0), (1, 2, 777, 4096, 1, 1.0),
                                     (1, 2, 512, 4100, 3, 1.0), (2, 2, 300, 2049, 2, 1.0), (1, 2, 256, 640, 1, 4.0),
                                     (1, 1, 256, 9000, 1, 1.0)]:
        q = torch.randn(B, Lq, H, 128, device=dev, generator=g)
        k = torch.randn(B, Lk, H, 128, device=dev, generator=g)
        v = torch.randn(B, Lk, H, 128, device=dev, generator=g)
        # scale > 1: growing score range along the keys (exercises the running-max moves)
        k = k * torch.linspace(0.2, scale, Lk, device=dev).view(1, Lk, 1, 1)
        q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
        ref = torch.softmax(torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * 128 ** -0.5, -1)
        ref = torch.einsum("bhqk,bkhd->bqhd", ref, v.float())
        nb = (q.float().norm(dim=-1).max().item(), k.float().norm(dim=-1).max().item())
        for bounds in (None, nb):  # online max, bounded shift
            out = N.attn_fwd(q, k, v, n_split=ns, norm_bounds=bounds).float()
            rel = float((out - ref).norm() / ref.norm())
            ok = rel < 4e-3 and bool(torch.isfinite(out).all())
            bad += not ok
            print(json.dumps({"B": B, "H": H, "Lq": Lq, "Lk": Lk, "split": ns, "scale": scale,
                              "bounded": bounds is not None, "rel_l2": rel, "ok": ok}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
