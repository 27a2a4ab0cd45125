set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_dit_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error" gpurun_out/fp8_tests.log | tail -12; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py --linear-precision fp8 --no-cpu-baseline > gpurun_out/bench_fp8.log 2> gpurun_out/bench_fp8.err
rc=$?; tail -n 1 gpurun_out/bench_fp8.log | cut -c1-900; exit $rc
