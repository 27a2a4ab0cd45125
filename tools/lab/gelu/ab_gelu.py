"""Lab A/B: the MLP1 + GELU epilogue by LDS table (the product, libcp25.so) vs exact-erf GELU in
VALU on every element (tools/lab/gelu/libcp25_gelu_valu.so, -DCP25_LAB_GELU_VALU), at the metric shape (M = 218 240,
N = 8192, K = 2048), alternating in one process; plus the plain MLP1 GEMM for the epilogue's cost, and the VALU
epilogue over every finite bf16 value against cp25_gelu (bit-identity). One JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

dev = torch.device("cuda:0")
lab = ctypes.CDLL(os.path.join(ROOT, "tools/lab/gelu/libcp25_gelu_valu.so"))
lab.cp25_gemm_epi.argtypes = N.SIGNATURES["cp25_gemm_epi"]


def lab_gemm(a, w, out, epi):
    rc = lab.cp25_gemm_epi(a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0),
                           a.shape[0], w.shape[0], a.shape[1], epi, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    return out


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


N.load_library()
only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None  # one form (the PMC passes)
if only:
    M, Nn, K = 218240, 8192, 2048
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
    out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    fn = (lambda: N.gemm_epi(x, w, epilogue=N.EPI_GELU, out=out)) if only == "table" else \
        (lambda: lab_gemm(x, w, out, N.EPI_GELU))
    print(json.dumps({"only": only, "ms": timed(fn, iters=2)}))
    sys.exit(0)
# bit-identity of the VALU epilogue over every finite bf16 value
bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
xv = bits[torch.isfinite(bits.float())].to(dev)
a = torch.zeros(xv.numel(), 2048, dtype=torch.bfloat16, device=dev)
a[:, 0] = xv
w1 = torch.zeros(256, 2048, dtype=torch.bfloat16, device=dev)
w1[:, 0] = 1.0
ref = xv.clone()
N.gelu_(ref)
g_lab = lab_gemm(a, w1, torch.empty(xv.numel(), 256, dtype=torch.bfloat16, device=dev), N.EPI_GELU)
g_prod = N.gemm_epi(a, w1, epilogue=N.EPI_GELU)
rec = {"valu_equal_cp25_gelu_all_bf16": bool(torch.equal(g_lab, ref[:, None].expand(-1, 256))),
       "table_equal_cp25_gelu_all_bf16": bool(torch.equal(g_prod, ref[:, None].expand(-1, 256)))}
del a, g_lab, g_prod

M, Nn, K = 218240, 8192, 2048
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
w = (torch.randn(Nn, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
res = {"table": [], "valu": [], "plain": []}
for r in range(4):
    order = ("table", "valu") if r % 2 == 0 else ("valu", "table")
    for f in order:
        if f == "table":
            res[f].append(round(timed(lambda: N.gemm_epi(x, w, epilogue=N.EPI_GELU, out=out)), 4))
        else:
            res[f].append(round(timed(lambda: lab_gemm(x, w, out, N.EPI_GELU)), 4))
    res["plain"].append(round(timed(lambda: N.gemm_epi(x, w, out=out)), 4))
rec.update({f + "_ms": v for f, v in res.items()})
rec.update({f + "_min_ms": min(v) for f, v in res.items()})
print(json.dumps(rec), flush=True)
