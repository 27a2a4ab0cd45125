set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python tools/sim_cp_rank.py --cp 1 2 4 8 > gpurun_out/sim_cp.log 2>&1 && \
timeout -k 10 300 python tools/sim_cp_rank.py --cp 8 --gather expand >> gpurun_out/sim_cp.log 2>&1
rc=$?; grep -E "passed|failed|rel-L2 \(CP" gpurun_out/gpu_tests.log; grep '{' gpurun_out/sim_cp.log; exit $rc
