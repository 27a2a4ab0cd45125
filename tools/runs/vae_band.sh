set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python tools/sim_vae_band.py > gpurun_out/sim_vae.log 2>&1
rc=$?; grep -E "passed|failed|banded" gpurun_out/gpu_tests.log; grep '{' gpurun_out/sim_vae.log; exit $rc
