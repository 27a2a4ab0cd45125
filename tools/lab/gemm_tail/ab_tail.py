"""Lab A/B: the bf16 block GEMMs with the tail row-slice plan (libcp25.so) against the whole-tile
plan (tools/lab/gemm_tail/libcp25_base.so, gemm.hip before it), alternating in one process, at a CP = 8 lane's M
(13 640 = 109 120 / 8 tokens x B 1), the CP = 8 rank's whole batch (27 280), config 5's (9 600) and the metric's
(218 240); plus each output against the other (bit-identical). One JSON line per shape."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

dev = torch.device("cuda:0")
base = ctypes.CDLL(os.path.join(ROOT, "tools/lab/gemm_tail/libcp25_base.so"))
base.cp25_gemm_epi.argtypes = N.SIGNATURES["cp25_gemm_epi"]


def base_gemm(a, w, out, epi):
    rc = base.cp25_gemm_epi(a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0),
                            a.shape[0], w.shape[0], a.shape[1], epi, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    return out


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


N.load_library()
g = torch.Generator(device=dev).manual_seed(0)
for M in (13640, 27280, 9600, 218240):
    for name, Nn, K, epi in (("qkv", 6144, 2048, 0), ("proj", 2048, 2048, 0), ("mlp1_gelu", 8192, 2048, 1),
                             ("mlp2", 2048, 8192, 0)):
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(Nn, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        o1 = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        o2 = torch.empty_like(o1)
        N.gemm_epi(x, w, epilogue=epi, out=o1)
        base_gemm(x, w, o2, epi)
        same = bool(torch.equal(o1, o2))
        t = {"slices": [], "base": []}
        for r in range(4):
            for f in (("slices", "base") if r % 2 == 0 else ("base", "slices")):
                t[f].append(round(timed(lambda: N.gemm_epi(x, w, epilogue=epi, out=o1)) if f == "slices" else
                                  timed(lambda: base_gemm(x, w, o2, epi)), 4))
        tiles = -(-M // 256) * (Nn // 256)
        print(json.dumps({"M": M, "gemm": name, "N": Nn, "K": K, "tiles": tiles, "bit_identical": same,
                          "slices_ms": t["slices"], "base_ms": t["base"], "slices_min": min(t["slices"]),
                          "base_min": min(t["base"]), "speedup": min(t["base"]) / min(t["slices"])}), flush=True)
        del x, w, o1, o2
