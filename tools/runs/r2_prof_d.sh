# rocprofv3 kernel trace + stats of the bench (current build), plus the GPU busy / gap analysis of the trace
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r2d
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2d -o bench -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r2d_bench.log 2>&1
rc=$?; tail -c 400 gpurun_out/prof_r2d_bench.log
[ $rc -eq 0 ] || exit $rc
find gpurun_out/prof_r2d -name "*.csv" | head
python3 tools/trace_gaps.py $(find gpurun_out/prof_r2d -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_r2d/gaps.txt
cat gpurun_out/prof_r2d/gaps.txt
