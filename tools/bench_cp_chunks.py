"""Attention cost of one context-parallel rank's self-attention under the K/V head-chunk pipeline.

Simulates rank 0 of CP = N at the metric shape (queries = L/N local tokens, keys = all L gathered
tokens, B = 2, H = 16) with the gathered K/V already resident, and times (HIP events, same process,
interleaved rounds) the attention work of one block:
  full   : one launch over all heads (what a non-pipelined all-gather would run);
  serial : nc head-chunk launches on one stream (n_split = library plan, or --split);
  streams: nc head-chunk launches on nc streams (the dispatcher fills one chunk's tail with the
           next chunk's workgroups).
usage: python tools/bench_cp_chunks.py [--cp 8] [--nc 4] [--rounds 3]
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
    ap.add_argument("--cp", type=int, default=8)
    ap.add_argument("--nc", type=int, default=4)
    ap.add_argument("--L", type=int, default=109120)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--split", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, H, hd = 2, 16, 128
    n = a.L // a.cp
    Hc = H // a.nc
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(n, B, H, hd, device=dev, generator=g).to(torch.bfloat16)
    kv = [torch.randn(a.L * B, 2 * Hc * hd, device=dev, generator=g).to(torch.bfloat16) for _ in range(a.nc)]
    o = torch.empty(n, B, H, hd, device=dev, dtype=torch.bfloat16)
    kf = torch.randn(a.L, B, H, hd, device=dev, generator=g).to(torch.bfloat16)
    vf = torch.randn(a.L, B, H, hd, device=dev, generator=g).to(torch.bfloat16)
    streams = [torch.cuda.Stream(device=dev) for _ in range(a.nc)]
    main_s = torch.cuda.current_stream()

    def views(c):
        kc = kv[c].view(a.L, B, 2, Hc, hd)
        return kc[:, :, 0].transpose(0, 1), kc[:, :, 1].transpose(0, 1)

    def chunk(c, ns):
        k, v = views(c)
        N.attn_fwd(q[:, :, c * Hc:(c + 1) * Hc].transpose(0, 1), k, v,
                   out=o[:, :, c * Hc:(c + 1) * Hc].transpose(0, 1), n_split=ns)

    ns_chunk = a.split or N.attn_plan(B, Hc, n, a.L)

    def run_full():
        N.attn_fwd(q.transpose(0, 1), kf.transpose(0, 1), vf.transpose(0, 1), out=o.transpose(0, 1), n_split=1)

    def run_serial():
        for c in range(a.nc):
            chunk(c, ns_chunk)

    def run_streams():
        ev = torch.cuda.Event()
        ev.record(main_s)
        for c in range(a.nc):
            streams[c].wait_event(ev)
            with torch.cuda.stream(streams[c]):
                chunk(c, 1)
        for c in range(a.nc):
            main_s.wait_stream(streams[c])

    variants = {"full": run_full, "serial": run_serial, "streams": run_streams}
    res = {k: [] for k in variants}
    for f in variants.values():
        f()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, f in variants.items():
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            f()
            e1.record(main_s)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1))
    flop = 4.0 * B * H * n * a.L * hd
    out = {"cp": a.cp, "nc": a.nc, "Lq": n, "Lk": a.L, "chunk_split": ns_chunk}
    for k, v in res.items():
        ms = sorted(v)[len(v) // 2]
        out[k + "_ms"] = ms
        out[k + "_tflops"] = flop / ms / 1e9
    print(json.dumps(out))


if __name__ == "__main__":
    main()
