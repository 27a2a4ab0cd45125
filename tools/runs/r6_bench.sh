#!/bin/bash
# round 6: the driver's bench command on the current tree, then the same command under rocprofv3 --kernel-trace --stats
# (the summary profiles/r6/bench_<x>/ keeps); $1 names the run
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r6bench_${1:-a}
mkdir -p $O
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', round(d['ms_per_step'], 1), 'attn ms', round(d['roofline']['avg_launch_ms'], 2), 'frac', round(d['roofline']['frac'], 4))
print('trained', json.dumps(d.get('trained_norm_weights')))
print('cpu', json.dumps(d.get('cpu_baseline')))"
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
  python3 tools/prof_db_stats.py $(find $O/prof -name "*.db" | head -1) $O/bench_kernel_stats.csv
  head -8 $O/bench_kernel_stats.csv | cut -c1-160
fi
