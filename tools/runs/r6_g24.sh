#!/bin/bash
# round 6, final tree: rehearsal of the self-launched multi-rank bench flow on one GPU (gloo ranks sharing cuda:0):
# 2 ranks over a whole 3-step video, then 4 ranks with the per-evaluation model (no whole video)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r6g24
mkdir -p $O
timeout -k 10 900 python bench.py --gpus 2 --backend gloo --share-device --steps 2 --warmup 1 --num-steps 3 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -30 $O/bench_gloo2.err; exit 1; }
tail -1 $O/bench_gloo2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['value_method'], json.dumps(d.get('context_parallel'))[:400])"
timeout -k 10 900 python bench.py --gpus 4 --backend gloo --share-device --steps 2 --warmup 1 --num-steps 3 --no-whole-video > $O/bench_gloo4.json 2> $O/bench_gloo4.err || { tail -30 $O/bench_gloo4.err; exit 1; }
tail -1 $O/bench_gloo4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['value_method'], json.dumps(d.get('context_parallel'))[:400])"
