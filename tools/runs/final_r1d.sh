set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -n 1 gpurun_out/smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline --linear-precision fp8 > gpurun_out/benchfull_fp8.log 2> gpurun_out/benchfull_fp8.err
rc=$?; python3 -c "import json; j=json.loads(open('gpurun_out/benchfull_fp8.log').read().strip().splitlines()[-1]); print('fp8', j['value'], j['ms_per_step'], j['roofline']['avg_launch_ms'])"; exit $rc
