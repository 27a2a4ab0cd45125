set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/attn1d_ab2.log
for i in 1 2; do
  for v in 2w:dmabuf 1d:dmabuf 1d:dmaglobal; do
    CP25_ATTN_KERNEL=${v%%:*} timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 3 --lib tools/lab/libcp25_${v##*:}.so >> gpurun_out/attn1d_ab2.log 2>&1 || exit 1
    echo "variant $v" >> gpurun_out/attn1d_ab2.log
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/attn1d_ab2.log'):
    if l.startswith('{'): d=json.loads(l)
    elif l.startswith('variant'): print(l.split()[1], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])
PY
