"""Same-box A/B at the metric self-attention shape (B 2, H 16, L 109 120): cp25_attn_fwd_bounded on q vs
cp25_attn_fwd_prescaled on q * scale * log2(e) (the fp8 option's form). HIP events; one JSON line each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

dev = torch.device("cuda:0")
B, H, D, L = 2, 16, 128, 109120
g = torch.Generator(device=dev).manual_seed(0)


def rms_rows():
    x = torch.randn(B, L, H, D, device=dev, generator=g)
    return (x / x.pow(2).mean(-1, keepdim=True).sqrt()).to(torch.bfloat16)


q, k, v = rms_rows(), rms_rows(), torch.randn(B, L, H, D, device=dev, generator=g).to(torch.bfloat16)
c = D ** -0.5 * 1.4426950408889634
qs = (q.float() * c).to(torch.bfloat16)
bnd = D ** 0.5 * 1.02
out = torch.empty_like(q)
runs = {"bounded": lambda: N.attn_fwd(q, k, v, out=out, norm_bounds=(bnd, bnd)),
        "prescaled": lambda: N.attn_fwd(qs, k, v, out=out, norm_bounds=(bnd * c, bnd), prescaled=True)}
flop = 4.0 * B * H * L * L * D
for rnd in range(3):
    for name, fn in runs.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(2):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 2
        print(json.dumps({"round": rnd, "kernel": name, "ms": ms, "tflops": flop / ms / 1e9}), flush=True)
