#!/bin/bash
# round 4: the driver's bench command (whole video timed), rocprofv3 kernel stats of a shorter bench, the trained-size
# norm-weight runs, and the PMC passes of the self-attention at the bench shape
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { tail $O/bench_driver_cmd.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_driver_cmd.json').read().strip().splitlines()[-1])
print(d['value'], d['modeled_value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-whole-video > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
python3 tools/rocpd_stats.py $O/prof/run_results.db > $O/bench_kernel_stats.csv && head -8 $O/bench_kernel_stats.csv | cut -c1-160
for nw in "" "0.5,3"; do
  tag=${nw:-unit}
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-whole-video ${nw:+--norm-weights $nw} > $O/bench_nw_$tag.json 2> $O/bench_nw_$tag.err || { tail $O/bench_nw_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_nw_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['attention_kernels'])"
done
bash tools/pmc_passes.sh $O/pmc_self python3 tools/bench_attn.py --iters 1 --bounded --fused --prescaled || exit 1
python3 tools/pmc_summary.py $O/pmc_self > $O/pmc_self.json && cat $O/pmc_self.json
