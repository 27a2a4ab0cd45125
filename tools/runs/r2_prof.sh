# rocprofv3 kernel stats of the driver bench command (fewer steps) + PMC passes of the self-attention
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2 -o bench -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r2_bench.log 2>&1
rc=$?; tail -c 600 gpurun_out/prof_r2_bench.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 bash tools/pmc_attn.sh gpurun_out/pmc_r2 && python3 tools/pmc_summary.py gpurun_out/pmc_r2 > gpurun_out/pmc_r2/SUMMARY.json && cat gpurun_out/pmc_r2/SUMMARY.json
