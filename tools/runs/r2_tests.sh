set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2.log 2>&1
rc=$?; tail -n 5 gpurun_out/gpu_tests_r2.log; exit $rc
