set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_vae_attn_gpu.py tests/test_vae_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error|assert" gpurun_out/conv_tests.log | tail -16; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/bench_conv.py > gpurun_out/conv_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/conv_bench.log; [ $rc = 0 ] || exit $rc
rm -rf gpurun_out/pmc_conv
bash tools/pmc_conv.sh gpurun_out/pmc_conv && python3 tools/pmc_conv_summary.py gpurun_out/pmc_conv > gpurun_out/pmc_conv/SUMMARY.json && cat gpurun_out/pmc_conv/SUMMARY.json
