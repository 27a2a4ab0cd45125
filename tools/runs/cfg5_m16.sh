# config 5 (action-conditioned AR 512f, 480x640) with the 16x16x32 attention: bf16 (m16 vs d128), fp8 GEMMs, all fp8
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/cfg5m
timeout -k 10 300 python tools/bench_action_ar.py > gpurun_out/cfg5m/bf16_m16.json 2> gpurun_out/cfg5m/e1.err && \
CP25_ATTN_MFMA=32 timeout -k 10 300 python tools/bench_action_ar.py > gpurun_out/cfg5m/bf16_d128.json 2> gpurun_out/cfg5m/e2.err && \
timeout -k 10 300 python tools/bench_action_ar.py --linear-precision fp8 > gpurun_out/cfg5m/fp8_gemm_m16.json 2> gpurun_out/cfg5m/e3.err && \
timeout -k 10 300 python tools/bench_action_ar.py --linear-precision fp8 --attention-precision fp8 > gpurun_out/cfg5m/fp8_all.json 2> gpurun_out/cfg5m/e4.err
rc=$?; [ $rc = 0 ] || exit $rc
tail -n1 gpurun_out/cfg5m/*.json | cut -c1-300

rm -f gpurun_out/cfg5m/vb128_ab.log
for i in 1 2; do
  for n in base vb128; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 --lib tools/lab/libcp25_$n.so >> gpurun_out/cfg5m/vb128_ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*' gpurun_out/cfg5m/vb128_ab.log | paste - -
