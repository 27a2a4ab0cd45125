# fp8-attention emulation A/B: the DiT self-attention kernel with half of its QK^T and/or P.V MFMAs (and their
# operand reads) removed, the work an fp8 operand would save; interleaved rounds, same box
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/fp8emu_ab.log
for i in 1 2; do
  for n in base qkhalf pvhalf both; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 --lib tools/lab/libcp25_fp8emu_$n.so >> gpurun_out/fp8emu_ab.log 2>&1 || exit 1
  done
done
cut -c1-60,230-420 gpurun_out/fp8emu_ab.log
