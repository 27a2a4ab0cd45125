# round-2 m16 build: attention PMC passes (HBM traffic prior), the driver's bench command, rocprofv3 kernel stats
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out/r2f
bash tools/pmc_attn.sh gpurun_out/r2f/pmc && python3 tools/pmc_summary.py gpurun_out/r2f/pmc > gpurun_out/r2f/pmc/SUMMARY.json || exit 1
cat gpurun_out/r2f/pmc/SUMMARY.json
timeout -k 10 560 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2f/bench_driver_cmd.json 2> gpurun_out/r2f/bench_driver_cmd.err || exit 1
tail -1 gpurun_out/r2f/bench_driver_cmd.json | cut -c1-600
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r2f/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/r2f/bench_prof.json 2> gpurun_out/r2f/bench_prof.err || exit 1
find gpurun_out/r2f/prof -name "*kernel_stats.csv" | head -3
