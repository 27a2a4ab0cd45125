#!/bin/bash
# round 5: rehearsal of the self-launched multi-rank bench flow on one GPU (2 gloo ranks sharing cuda:0)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5g2${1:-}
mkdir -p $O
timeout -k 10 900 python bench.py --gpus 2 --backend gloo --share-device --steps 2 --warmup 1 --num-steps 3 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -30 $O/bench_gloo2.err; exit 1; }
tail -1 $O/bench_gloo2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['value_method'], json.dumps(d.get('context_parallel'))[:400])"
