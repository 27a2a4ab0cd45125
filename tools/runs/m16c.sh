# m16 attention lab A/B at the metric shape (prescaled): row sums by MFMA, early loads, read-ahead depth
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16c
rm -f gpurun_out/m16c/ab.log
for i in 1 2; do
  CP25_ATTN_MFMA=32 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/m16c/ab.log 2>&1 || exit 1
  for lib in "" tools/lab/libcp25_lsum.so tools/lab/libcp25_lsumearly.so tools/lab/libcp25_ahead2.so tools/lab/libcp25_lsum2.so; do
    CP25_ATTN_MFMA=16 timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 ${lib:+--lib $lib} >> gpurun_out/m16c/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*\|"check_rel_l2": [0-9.e-]*' gpurun_out/m16c/ab.log | paste - - -
