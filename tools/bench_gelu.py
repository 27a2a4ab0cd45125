"""cp25_gelu throughput at the DiT's MLP hidden shape [218240, 8192] bf16 (in place, HIP events).

usage: python tools/bench_gelu.py [--lib tools/lab/libcp25_x.so]
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
    x = torch.randn(218240, 8192, device="cuda").to(torch.bfloat16)
    N.gelu_(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        N.gelu_(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(json.dumps({"lib": os.path.basename(a.lib) or "libcp25.so", "ms": ms, "TBps": 4 * x.numel() / ms / 1e9}))


if __name__ == "__main__":
    main()
