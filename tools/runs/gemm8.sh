set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k "not nothing" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error|assert" gpurun_out/gemm_tests.log | tail -14; [ $rc = 0 ] || exit $rc
GEMM_LABS=16,64 timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/gemm_bench.log; exit $rc
