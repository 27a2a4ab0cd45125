#!/bin/bash
# round 5: the driver's bench command on the final tree, then rocprofv3 kernel stats of a shorter bench
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r5f${1:-a}
mkdir -p $O
timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { tail $O/bench_driver_cmd.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_driver_cmd.json').read().strip().splitlines()[-1])
print(d['value'], d['modeled_value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])
print(json.dumps(d.get('trained_norm_weights')))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-whole-video --trained-evals 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
python3 tools/rocpd_stats.py $O/prof/run_results.db > $O/bench_kernel_stats.csv && head -12 $O/bench_kernel_stats.csv | cut -c1-160
