"""cp25_gelu_quant_fp8 / cp25_quant_fp8_rows throughput at the DiT's shapes (HIP events); one JSON line
per shape: ms per launch and GB/s of algorithmic traffic (2 B read + 1 B written per element)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402

if len(sys.argv) > 2 and sys.argv[1] == "--lib":  # lab build of libcp25.so (same-box A/B)
    N._LIB_PATH = sys.argv[2]
dev = torch.device("cuda:0")
for M, K, gelu in [(218240, 8192, True), (218240, 2048, False), (9600, 8192, True), (9600, 2048, False)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    for _ in range(2):
        N.quant_fp8_rows(x, gelu=gelu)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    e0.record()
    for _ in range(it):
        N.quant_fp8_rows(x, gelu=gelu)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(json.dumps({"lib": os.path.basename(N.library_path()), "M": M, "K": K, "gelu": gelu, "ms": ms, "GB_s": 3.0 * M * K / ms / 1e6}), flush=True)
    del x
    torch.cuda.empty_cache()
