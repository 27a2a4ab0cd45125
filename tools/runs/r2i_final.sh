# final tree: full GPU suite + smoke, the driver's bench command, rocprofv3 kernel stats of a shorter bench
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out/r2i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r2i/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r2i/gpu_tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r2i/gpu_tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2i/smoke.log 2>&1 || { tail -20 gpurun_out/r2i/smoke.log; exit 1; }
tail -1 gpurun_out/r2i/smoke.log
timeout -k 10 560 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2i/bench_driver_cmd.json 2> gpurun_out/r2i/bench_driver_cmd.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r2i/bench_driver_cmd.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config']['seconds_per_video'], d['roofline']['avg_launch_ms'], d['roofline']['achieved'], d['roofline']['frac'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r2i/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/r2i/bench_prof.json 2> gpurun_out/r2i/bench_prof.err || exit 1
python3 tools/rocpd_stats.py gpurun_out/r2i/prof/run_results.db > gpurun_out/r2i/bench_kernel_stats.csv && head -4 gpurun_out/r2i/bench_kernel_stats.csv | cut -c1-160
