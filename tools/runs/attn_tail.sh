# attention tail quantization: L = 109120 (13 664 workgroups = 53.4 rounds of 256) vs 108544 (53 rounds) vs 110592 (54)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/attn_tail.log
for i in 1 2; do
  for L in 108544 109120 110592; do
    timeout -k 10 120 python tools/bench_attn.py --L $L --fused --bounded --prescaled --iters 3 >> gpurun_out/attn_tail.log 2>&1 || exit 1
  done
done
grep -o '"Lq": [0-9]*\|"ms": [0-9.]*' gpurun_out/attn_tail.log | paste - -
