set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2.log 2>&1
rc=$?; tail -n 4 gpurun_out/gpu_tests_r2.log; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r2.log 2> gpurun_out/bench_r2.err
rc=$?; tail -c 1500 gpurun_out/bench_r2.log; exit $rc
