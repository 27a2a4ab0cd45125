set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/vae_tests.log 2>&1 && \
timeout -k 10 200 python tools/sim_vae_band.py --cp 1 8 > gpurun_out/vae_perf.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed" gpurun_out/vae_tests.log; grep '{' gpurun_out/vae_perf.log; exit $rc
