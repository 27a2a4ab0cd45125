# GELU epilogue routing + m16 attention: parity tests, GEMM A/B, attention PMC, MLP1 A/B at the metric geometry,
# the driver's bench command and a rocprofv3 kernel-stats run
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out/r2g
timeout -k 10 500 python -u -m pytest tests/test_dit_ops_gpu.py tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_dit_gpu.py tests/test_parity_depth_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r2g/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r2g/tests.log | tail -30; exit 1; }
grep -E "passed|failed|truth" gpurun_out/r2g/tests.log | tail -8
GEMM_LABS= timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/r2g/gemm_bench.log 2>&1 || exit 1
grep mlp1 gpurun_out/r2g/gemm_bench.log | cut -c1-400
bash tools/pmc_attn.sh gpurun_out/r2g/pmc && python3 tools/pmc_summary.py gpurun_out/r2g/pmc > gpurun_out/r2g/pmc/SUMMARY.json || exit 1
cat gpurun_out/r2g/pmc/SUMMARY.json
for m in lib own; do
  CP25_MLP1_GEMM=$m timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r2g/mlp1_$m.json 2> gpurun_out/r2g/mlp1_$m.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r2g/mlp1_$m.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 560 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2g/bench_driver_cmd.json 2> gpurun_out/r2g/bench_driver_cmd.err || exit 1
tail -1 gpurun_out/r2g/bench_driver_cmd.json | cut -c1-700
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r2g/prof -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/r2g/bench_prof.json 2> gpurun_out/r2g/bench_prof.err || exit 1
find gpurun_out/r2g/prof -name "*kernel_stats.csv" | head -3
