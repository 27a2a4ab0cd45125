set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -n 1 gpurun_out/smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python bench.py > gpurun_out/bench_final.log 2> gpurun_out/bench_final.err
rc=$?; tail -n 1 gpurun_out/bench_final.log | cut -c1-1500; exit $rc
