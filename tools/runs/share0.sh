# CFG block-0 sharing: DiT tests (shared path exercised by every sampler test), then the metric bench
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dit_gpu.py tests/test_inference_gpu.py tests/test_parity_depth_gpu.py tests/test_action_gpu.py tests/test_multiview_gpu.py -x -v -s \
  --timeout 300 --timeout-method thread > gpurun_out/share0_tests.log 2>&1 || { tail -40 gpurun_out/share0_tests.log; exit 1; }
grep -E "shared block-0|rel-L2|hip-vs-truth|passed|failed" gpurun_out/share0_tests.log
timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/share0_bench.json 2> gpurun_out/share0_bench.err
tail -c 1500 gpurun_out/share0_bench.json
