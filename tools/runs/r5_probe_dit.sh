#!/bin/bash
# round 5: the self-attention's anatomy inside the DiT (unit vs trained-size q/k norm weights), then the same kernel
# forms isolated (tools/bench_attn.py) on the same box, for the in-bench cost of trained-size weights
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5pdit
mkdir -p $O
timeout -k 10 400 python3 tools/probe_in_dit.py > $O/in_dit.log 2> $O/in_dit.err || { tail $O/in_dit.err; exit 1; }
grep -E "^(unit|trained)" $O/in_dit.log | cut -c1-400
B="python3 tools/bench_attn.py --fused --bounded --prescaled --qnorm --iters 3 --lib tools/lab/libcp25_probe.so --probe 800"
for w in "1,1" "0.5,3"; do
  timeout -k 10 120 $B --wrange $w >> $O/isolated.jsonl 2>>$O/err.log || exit 1
done
python3 -c "
import json
for l in open('$O/isolated.jsonl'):
    d=json.loads(l); p=d['probe']; print('isolated', d['wrange'], round(d['ms'],2), p['period'], p['clock_ghz'], p.get('rescale_tiles_per_wave'))"
