# phase anatomy (s_memtime) of the m16 vs d128 attention kernels, bounded form, metric length
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16probe
for i in 1 2; do
  CP25_ATTN_MFMA=32 timeout -k 10 120 python tools/attn_probe.py --L 109120 --bounded --t0 600 >> gpurun_out/m16probe/probe.log 2>&1 || exit 1
  CP25_ATTN_MFMA=16 timeout -k 10 120 python tools/attn_probe.py --L 109120 --bounded --t0 600 >> gpurun_out/m16probe/probe.log 2>&1 || exit 1
done
grep '^{' gpurun_out/m16probe/probe.log
rm -f gpurun_out/m16probe/ab.log
for i in 1 2; do
  CP25_ATTN_MFMA=32 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/m16probe/ab.log 2>&1 || exit 1
  for lib in "" tools/lab/libcp25_tile0.so tools/lab/libcp25_early.so; do
    CP25_ATTN_MFMA=16 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 ${lib:+--lib $lib} >> gpurun_out/m16probe/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*' gpurun_out/m16probe/ab.log | paste - -
timeout -k 10 300 python -u -m pytest tests/test_attn_m16_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/m16probe/tests.log 2>&1 || { grep -E "m16|PASS|FAIL|Error|assert" gpurun_out/m16probe/tests.log | tail -30; exit 1; }
grep -E "^m16|passed|failed" gpurun_out/m16probe/tests.log
