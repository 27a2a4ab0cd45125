#!/bin/bash
# round 5: the fp32 conditioning GEMM (cp25_gemm_f32) and the per-prompt context on the hand-written GEMMs: their
# tests, the DiT/oracle parity tests that now run through them, and the final linear timed against the library
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5f32
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gemm_f32_gpu.py \
  > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|gemm_f32|bias-column|rel-L2" $O/tests.log | tail -40
[ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 120 python3 - <<'PY'
import sys; sys.path.insert(0, "cosmos-predict2.5_amd")
import torch, torch.nn.functional as F
from cosmos_predict2 import _native as N
dev = torch.device("cuda:0")
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / it
x = torch.randn(218240, 2048, device=dev); w = torch.randn(64, 2048, device=dev)
for name, fn in (("library", lambda: F.linear(x, w)), ("cp25_gemm_f32", lambda: N.gemm_f32(x, w))):
    ms = t(fn)
    print("final linear", name, round(ms, 4), "ms", round(2 * 218240 * 64 * 2048 / ms / 1e9, 1), "TF/s",
          round((x.numel() + w.numel() + 218240 * 64) * 4 / ms / 1e6, 1), "GB/s")
for (M, Nn, K) in ((62, 2048, 2048), (62, 6144, 2048), (62, 21504, 2048), (62, 256, 2048), (62, 4096, 256)):
    a = torch.randn(M, K, device=dev); b = torch.randn(Nn, K, device=dev)
    print("fp32", M, Nn, K, "library", round(t(lambda: F.linear(a, b)), 4), "own", round(t(lambda: N.gemm_f32(a, b)), 4), "ms")
a1 = torch.randn(62, 84 * 256, device=dev).view(62, 84, 256).transpose(0, 1); w2 = torch.randn(84, 6144, 256, device=dev)
lo = torch.randn(62, 6144, device=dev)
print("ada2 batched library", round(t(lambda: torch.bmm(a1, w2.transpose(1, 2)) + lo), 4), "own",
      round(t(lambda: N.gemm_f32(a1, w2, add=lo)), 4), "ms")
PY
