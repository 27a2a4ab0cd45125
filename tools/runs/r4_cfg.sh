#!/bin/bash
# round 4: config 3 (14B Video2World semantics) and config 4 (480 x 832) tests, the zero-shift headroom test, then the
# driver's bench command (whole video by default now)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4cfg
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_configs_gpu.py tests/test_configs_net_gpu.py} \
  "tests/test_attn_m16_gpu.py::test_m16_zero_shift_top_of_window_long_keys" -m gpu -x -v -s --timeout 400 \
  --timeout-method thread > $O/tests${TAG}.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests${TAG}.log | tail -30; exit 1; }
grep -E "passed|failed|rel-L2|hip-|vs truth|forward|sampler" $O/tests${TAG}.log | tail -30
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
