# rocprofv3 kernel stats of the driver bench command (fewer steps)
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r2b
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2b -o bench -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r2b_bench.log 2>&1
rc=$?; tail -c 600 gpurun_out/prof_r2b_bench.log; exit $rc
