set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
CP25_ATTN_KERNEL=1d timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_attn_op_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn1d_tests.log 2>&1
rc=$?; tail -n 6 gpurun_out/attn1d_tests.log; [ $rc = 0 ] || exit $rc
rm -f gpurun_out/attn1d_ab.log
for i in 1 2; do
  for v in 2w 1w 1d; do
    CP25_ATTN_KERNEL=$v timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 >> gpurun_out/attn1d_ab.log 2>&1 || exit 1
    echo "variant $v" >> gpurun_out/attn1d_ab.log
  done
done
python3 - <<'PY'
import json
v=None
rows=[]
for l in open('gpurun_out/attn1d_ab.log'):
    if l.startswith('{'): d=json.loads(l)
    elif l.startswith('variant'): print(l.split()[1], round(d['ms'],2), round(d['tflops'],1), d['check_rel_l2'])
PY
