#!/bin/bash
# round 6: HIP-graph replay of the DiT forward (model.hip_graph): bit-identity tests, then config 5's AR loop eager vs
# graph, twice each in alternating order (same box)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r6_graph
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 600 python -u -m pytest tests/test_action_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for r in 1 2; do
  for g in "" "--hip-graph"; do
    if [ $r = 2 ]; then g=$([ -z "$g" ] && echo "--hip-graph" || echo ""); fi
    timeout -k 10 300 python tools/bench_action_ar.py $g ${ARGS:-} >> $O/ar.jsonl 2> $O/ar.err || { tail $O/ar.err; exit 1; }
    tail -n1 $O/ar.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['hip_graph'], d['frames_per_s'], d['s_per_chunk'])"
  done
done
