#!/bin/bash
# round 5: the driver's bench command on the current tree (+ the trained-norm-weights sub-record)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5bench_${1:-a}
mkdir -p $O
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', round(d['ms_per_step'], 1), 'attn ms', round(d['roofline']['avg_launch_ms'], 2), 'frac', round(d['roofline']['frac'], 4))
print('trained', json.dumps(d.get('trained_norm_weights')))
print('cpu', json.dumps(d.get('cpu_baseline')))"
