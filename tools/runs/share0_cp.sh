# CFG block-0 sharing in the CP lanes: CP=2 (two ranks on cuda:0 over gloo) vs CP=1, DiT tests
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_cp_gpu.py tests/test_dit_gpu.py tests/test_configs_gpu.py -x -v -s \
  --timeout 400 --timeout-method thread > gpurun_out/share0_cp.log 2>&1 || { tail -40 gpurun_out/share0_cp.log; exit 1; }
grep -E "CP=2|shared block-0|passed|failed" gpurun_out/share0_cp.log
