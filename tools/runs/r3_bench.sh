#!/bin/bash
# round 3: the driver's bench command, then rocprofv3 kernel stats of a shorter bench
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out/r3b
timeout -k 10 560 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b/bench_driver_cmd.json 2> gpurun_out/r3b/bench_driver_cmd.err || { tail gpurun_out/r3b/bench_driver_cmd.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3b/bench_driver_cmd.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config']['seconds_per_video'], d['roofline']['avg_launch_ms'], d['roofline']['achieved'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/r3b/bench_prof.json 2> gpurun_out/r3b/bench_prof.err || exit 1
python3 tools/rocpd_stats.py gpurun_out/r3b/prof/run_results.db > gpurun_out/r3b/bench_kernel_stats.csv && head -8 gpurun_out/r3b/bench_kernel_stats.csv | cut -c1-160
for nw in "" "0.5,3"; do
  tag=${nw:-unit}
  timeout -k 10 400 python bench.py --steps 4 --warmup 1 --no-cpu-baseline ${nw:+--norm-weights $nw} > gpurun_out/r3b/bench_nw_$tag.json 2> gpurun_out/r3b/bench_nw_$tag.err || { tail gpurun_out/r3b/bench_nw_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3b/bench_nw_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['attention_kernels'])"
done
