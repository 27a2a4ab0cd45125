"""Probe: fp8 (OCP e4m3fn) GEMMs through torch._scaled_mm (hipBLASLt) on gfx950 at the DiT's shapes,
tensor-wise and row-wise scales, vs bf16 F.linear; prints one JSON line per shape/mode."""
import json
import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
f8 = torch.float8_e4m3fn
FMAX = torch.finfo(f8).max


def t_ms(fn, it=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


M = 218240
for (N, K) in [(6144, 2048), (2048, 2048), (8192, 2048), (2048, 8192)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    ref = F.linear(a.float()[:4096], w.float())
    ms_bf = t_ms(lambda: F.linear(a, w))
    fl = 2 * M * N * K
    out = {"M": M, "N": N, "K": K, "bf16_ms": ms_bf, "bf16_tflops": fl / ms_bf / 1e9}
    # tensor-wise
    sa = a.abs().amax().float() / FMAX
    sw = w.abs().amax().float() / FMAX
    a8 = (a.float() / sa).to(f8)
    w8 = (w.float() / sw).to(f8)
    try:
        y = torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw, out_dtype=torch.bfloat16)
        out["tw_ms"] = t_ms(lambda: torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw, out_dtype=torch.bfloat16))
        out["tw_tflops"] = fl / out["tw_ms"] / 1e9
        out["tw_rel"] = ((y[:4096].float() - ref).norm() / ref.norm()).item()
    except Exception as e:  # noqa: BLE001
        out["tw_err"] = str(e)[:200]
    # row-wise
    ra = (a.abs().amax(dim=1, keepdim=True).float() / FMAX).clamp_min(1e-12)
    rw = (w.abs().amax(dim=1, keepdim=True).float() / FMAX).clamp_min(1e-12)
    a8r = (a.float() / ra).to(f8)
    w8r = (w.float() / rw).to(f8)
    try:
        y = torch._scaled_mm(a8r, w8r.t(), scale_a=ra, scale_b=rw.t(), out_dtype=torch.bfloat16)
        out["rw_ms"] = t_ms(lambda: torch._scaled_mm(a8r, w8r.t(), scale_a=ra, scale_b=rw.t(), out_dtype=torch.bfloat16))
        out["rw_tflops"] = fl / out["rw_ms"] / 1e9
        out["rw_rel"] = ((y[:4096].float() - ref).norm() / ref.norm()).item()
    except Exception as e:  # noqa: BLE001
        out["rw_err"] = str(e)[:200]
    print(json.dumps(out), flush=True)
    del a, w, a8, w8, a8r, w8r
    torch.cuda.empty_cache()
