set -o pipefail
export PYTHONUNBUFFERED=1
: > gpurun_out/ab_attn.log
timeout -k 10 120 python tools/check_attn_lib.py --lib tools/lab/libcp25_pk.so > gpurun_out/pk_check.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in base pk; do
    timeout -k 10 60 python tools/bench_attn.py --L 109120 --iters 3 --bounded --lib tools/lab/libcp25_$v.so 2>/dev/null | grep '{' >> gpurun_out/ab_attn.log || exit 1
  done
done
