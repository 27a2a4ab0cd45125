"""cp25_conv3d at the decoder's dominant shapes (704x1280 / 352x640 / 176x320, 3x3x3, 4 output frames): the halo
kernel (default) vs the per-tap kernel (cp25_conv3d_select(1)), HIP events, interleaved rounds in one process.
One JSON line per shape: ms and TFLOP/s (2 * 27 * Cin * Cout per output pixel). CONV_KINDS=halo,tap,halo4 picks the
kernels (halo: the 8-wave halo kernel, the default; halo4: the round-2 4-wave form, cp25_conv3d_select(2)); CONV_SHAPE=i one shape; ROUNDS=n;
CONV_LIB=path a lab build of libcp25.so (tools/lab/conv_variant.py) instead of the in-tree one."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402
from cosmos_predict2.vae import _Conv  # noqa: E402

if os.environ.get("CONV_LIB"):
    N._LIB_PATH = os.environ["CONV_LIB"]

dev = torch.device("cuda:0")
SHAPES = [(96, 96, 704, 1280), (192, 192, 352, 640), (384, 384, 176, 320), (384, 384, 88, 160)]
only = os.environ.get("CONV_SHAPE")


def timed(fn, iters=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters

for i, (cin, cout, H, W) in enumerate(SHAPES):
    if only is not None and only != str(i):
        continue
    g = torch.Generator(device=dev).manual_seed(i)
    frames = [torch.randn(H, W, cin, device=dev, generator=g).to(torch.bfloat16) for _ in range(6)]
    w = (torch.randn(cout, cin, 3, 3, 3, device=dev, generator=g) / (27 * cin) ** 0.5).to(torch.bfloat16)
    b = torch.zeros(cout, device=dev, dtype=torch.bfloat16)
    conv = _Conv(w, b, dev)
    run = lambda: conv(frames, 4, H, W, pad=(1, 1, 1, 1))  # noqa: E731
    modes = {"halo": 0, "tap": 1, "halo4": 2}
    kinds = os.environ.get("CONV_KINDS", "halo,tap").split(",")
    res = {k: [] for k in kinds}
    for _ in range(int(os.environ.get("ROUNDS", "2"))):
        for k in kinds:
            prev = N.conv3d_select(modes[k])
            res[k].append(timed(run))
            N.conv3d_select(prev)
    flop = 2.0 * 27 * cin * cout * H * W * 4
    rec = {"conv": f"{cin}->{cout} 3x3x3 {H}x{W} x4 frames"}
    for k in kinds:
        rec[f"{k}_ms"] = min(res[k])
        rec[f"{k}_tflops"] = flop / min(res[k]) / 1e9
    print(json.dumps(rec), flush=True)

# VAE AttentionBlock core at 704 x 1280 (88 x 160 = 14 080 tokens, one frame): cp25_vae_attn vs the round-1
# path (fp32 S by library GEMM, cp25_softmax_rows, library P V)
if only is None or only == "attn":
    from cosmos_predict2 import _native as N  # noqa: E402

    L, C = 88 * 160, 384
    g = torch.Generator(device=dev).manual_seed(9)
    qkv = torch.randn(1, L, 3 * C, device=dev, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]

    def old():
        s = torch.mm(q[0], k[0].t(), out_dtype=torch.float32)
        return torch.mm(N.softmax_rows(s, C ** -0.5), v[0].contiguous())

    t_new = min(timed(lambda: N.vae_attn(q, k, v)) for _ in range(2))
    t_old = min(timed(old) for _ in range(2))
    flop = 4.0 * L * L * C
    print(json.dumps({"vae_attn": f"L={L} d={C} one frame", "flash_ms": t_new, "round1_ms": t_old,
                      "flash_tflops": flop / t_new / 1e9, "round1_tflops": flop / t_old / 1e9}), flush=True)
