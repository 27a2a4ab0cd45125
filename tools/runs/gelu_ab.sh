set -o pipefail
export PYTHONUNBUFFERED=1
for r in 1 2; do for u in 1 2 4 8; do
  timeout -k 10 60 python tools/bench_gelu.py --lib tools/lab/libcp25_gu$u.so 2>/dev/null | grep '{' || exit 1
done; done
