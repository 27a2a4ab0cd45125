#!/bin/bash
# round 6: action tests, then config 5's AR loop (bf16) twice on the tree with the uint8 conditioning video
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_cfg5u8
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 600 python -u -m pytest tests/test_action_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for r in 1 2; do
  timeout -k 10 300 python tools/bench_action_ar.py >> $O/ar.jsonl 2> $O/ar.err || { tail $O/ar.err; exit 1; }
  tail -n1 $O/ar.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['frames_per_s'], d['s_per_chunk'])"
done
python3 - <<'PY' | tee $O/host_timing.txt
import time, numpy as np, torch, sys
sys.path.insert(0, "tests")
from test_action_cpu import _reference_form
from cosmos_predict2.action_conditioned import conditioning_video
img = np.random.RandomState(0).randint(0, 256, (480, 640, 3), dtype=np.uint8)
for name, f in (("reference fp32 round trip", _reference_form), ("uint8", conditioning_video)):
    ts = []
    for _ in range(5):
        t = time.perf_counter(); f(img, 13); ts.append((time.perf_counter() - t) * 1e3)
    print(f"{name}: {sorted(ts)[2]:.1f} ms per chunk (median of 5, {torch.get_num_threads()} threads)")
PY
