#!/bin/bash
# round 3 (session 2): the gated zero-shift / online attention pair with the data-tight key bound: tests, then the
# bench with q/k norm weights in [0.5, 3] (the gated pair) next to the unit weights
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3g
timeout -k 10 900 python -u -m pytest tests/test_attn_gated_gpu.py tests/test_parity_depth_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r3g/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3g/tests.log | head -20; tail -5 gpurun_out/r3g/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r3g/tests.log | tail -1
grep -E "gated|norm max" gpurun_out/r3g/tests.log | head
for nw in "0.5,3" "" "0.5,3"; do
  tag=${nw:-unit}
  timeout -k 10 400 python bench.py --steps 4 --warmup 1 --no-cpu-baseline ${nw:+--norm-weights $nw} > gpurun_out/r3g/bench_nw_$tag.json 2> gpurun_out/r3g/bench_nw_$tag.err || { tail gpurun_out/r3g/bench_nw_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3g/bench_nw_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['attention_kernels'])"
done
