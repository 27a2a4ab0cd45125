# m16 (+ MFMA row sums) as the default: GPU suite, then read-ahead / early-load A/B at the metric shape
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16e
rm -f gpurun_out/m16e/*.log
timeout -k 10 600 python -u -m pytest tests/test_xattn_persistent_gpu.py tests/test_attn_m16_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/m16e/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/m16e/gpu_tests.log | tail -30; exit 1; }
grep -E "passed|failed|truth" gpurun_out/m16e/gpu_tests.log | tail -12
for i in 1 2; do
  CP25_ATTN_MFMA=32 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/m16e/ab.log 2>&1 || exit 1
  for lib in "" tools/lab/libcp25_ahead4.so tools/lab/libcp25_ahead5.so tools/lab/libcp25_early.so; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 ${lib:+--lib $lib} >> gpurun_out/m16e/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*\|"check_rel_l2": [0-9.e-]*' gpurun_out/m16e/ab.log | paste - - -
