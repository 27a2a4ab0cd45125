"""Practical dense bf16 / fp8 MFMA ceiling of this MI355X: the vendor GEMM (hipBLASLt via torch) at large square
shapes, HIP events, random data (the chip's clock under sustained MFMA load is power-limited, so the spec peak
2.5 PF at 2.4 GHz is not reachable by any kernel; this is the reference point for the attention kernel's
roofline fraction). One JSON line per shape."""
import json

import torch


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    dev = torch.device("cuda:0")
    for n in (8192, 16384):
        a = torch.randn(n, n, device=dev).to(torch.bfloat16)
        b = torch.randn(n, n, device=dev).to(torch.bfloat16)
        c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
        ms = timed(lambda: torch.matmul(a, b.t(), out=c), 20 if n == 8192 else 6)
        print(json.dumps({"gemm": "bf16", "M": n, "N": n, "K": n, "ms": ms, "tflops": 2 * n ** 3 / ms / 1e9}), flush=True)
        a8, b8 = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
        one = torch.ones((), device=dev)
        ms = timed(lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16),
                   20 if n == 8192 else 6)
        print(json.dumps({"gemm": "fp8", "M": n, "N": n, "K": n, "ms": ms, "tflops": 2 * n ** 3 / ms / 1e9}), flush=True)
        a.zero_(), b.zero_()
        ms = timed(lambda: torch.matmul(a, b.t(), out=c), 20 if n == 8192 else 6)
        print(json.dumps({"gemm": "bf16 zeros", "M": n, "N": n, "K": n, "ms": ms, "tflops": 2 * n ** 3 / ms / 1e9}),
              flush=True)


if __name__ == "__main__":
    main()
