set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/ab_1w_lk.log
for lk in 4096 16384 109120; do
for k in 1w 2w; do
  CP25_ATTN_KERNEL=$k timeout -k 10 120 python tools/bench_attn.py --L 109120 --Lk $lk --bounded --prescaled --iters 4 > /tmp/o.txt 2>&1 || exit 1
  echo "Lk=$lk $k $(grep '^{' /tmp/o.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms"],2), round(d["tflops"]), d["check_rel_l2"])')" | tee -a gpurun_out/ab_1w_lk.log
done
done
