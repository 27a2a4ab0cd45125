set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_dit_ops_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/ops_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" gpurun_out/ops_tests.log | tail -6; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python - <<'PY'
import sys, torch
sys.path.insert(0, "cosmos-predict2.5_amd")
from cosmos_predict2 import _native as N
x = torch.randn(218240, 8192, device="cuda").to(torch.bfloat16)
N.gelu_(x); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): N.gelu_(x)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(f"gelu [218240, 8192]: {ms:.3f} ms, {2 * 2 * x.numel() / ms / 1e9:.2f} TB/s")
PY
