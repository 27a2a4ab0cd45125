"""Same-box A/B of one DiT block's six projections (QKV, self-out, cross-q, cross-out, MLP1, GELU +
MLP2) at the metric shape (M = 2 x 109 120 tokens, 2B widths): bf16 hipBLASLt GEMMs (+ cp25_gelu) vs
the fp8 path (cp25_quant_fp8_rows / cp25_gelu_quant_fp8 + hipBLASLt fp8 GEMMs). HIP events on the
current stream; prints one JSON line per precision."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2.dit import MinimalV1LVGDiT  # noqa: E402
from cosmos_predict2.net_config import tiny_dit  # noqa: E402

dev = torch.device("cuda:0")
M, D, F4 = 2 * 109120, 2048, 8192
net = MinimalV1LVGDiT(tiny_dit(), device=dev)
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
w = {k: (torch.randn(n, kk, device=dev, generator=g) * 0.02).to(torch.bfloat16)
     for k, (n, kk) in dict(qkv=(3 * D, D), o=(D, D), cq=(D, D), co=(D, D), l1=(F4, D), l2=(D, F4)).items()}


def block():
    net._linear(h, w["qkv"], "qkv")
    net._linear(h, w["o"], "o")
    net._linear(h, w["cq"], "cq")
    net._linear(h, w["co"], "co")
    u = net._linear(h, w["l1"], "l1")
    net._linear(u, w["l2"], "l2", gelu_in=True)


flop = 2 * M * D * (3 * D + 3 * D + 2 * F4)
for rnd in range(2):
    for prec in ("bf16", "fp8"):
        net.set_linear_precision(prec)
        for _ in range(2):
            block()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            block()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(json.dumps({"round": rnd, "precision": prec, "ms_per_block": ms, "tflops": flop / ms / 1e9}), flush=True)
