"""cp25_gemm_epi vs hipBLASLt (F.linear) at the DiT block projection shapes (M = 218 240 = 109 120 tokens x
CFG 2), HIP events; GELU fused vs linear + cp25_gelu. One JSON line per shape."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("GEMM_M", "218240"))


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for name, Nn, K in (("qkv", 6144, 2048), ("proj", 2048, 2048), ("mlp1", 8192, 2048), ("mlp2", 2048, 8192), ("k256", 2048, 256)):
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    flop = 2.0 * M * Nn * K
    t_lib = timed(lambda: torch.matmul(a, w.t(), out=out))
    os.environ["CP25_GEMM_KERNEL"] = "2ph"
    t_2ph = timed(lambda: N.gemm_epi(a, w, out=out))
    os.environ["CP25_GEMM_KERNEL"] = "8ph"
    t_own = timed(lambda: N.gemm_epi(a, w, out=out))
    t_lib2 = timed(lambda: torch.matmul(a, w.t(), out=out))
    labs = {}
    for lab in [x for x in os.environ.get("GEMM_LABS", "").split(",") if x]:
        os.environ["CP25_GEMM_KERNEL"] = "8ph_lab" + lab
        labs[lab] = timed(lambda: N.gemm_epi(a, w, out=out))
    os.environ["CP25_GEMM_KERNEL"] = "8ph"
    rec = {"gemm": name, "M": M, "N": Nn, "K": K, "hipblaslt_ms": [t_lib, t_lib2], "own_ms": t_own,
           "own_2ph_ms": t_2ph, "lab_ms": labs, "hipblaslt_tflops": flop / min(t_lib, t_lib2) / 1e9, "own_tflops": flop / t_own / 1e9}
    if name == "mlp1":
        def unfused():
            torch.matmul(a, w.t(), out=out)
            N.gelu_(out)
        rec["lib_plus_gelu_ms"] = timed(unfused)
        rec["own_gelu_fused_ms"] = timed(lambda: N.gemm_epi(a, w, epilogue=N.EPI_GELU, out=out))
    print(json.dumps(rec), flush=True)
