set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
CP25_ATTN_KERNEL=1w timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_attn_op_gpu.py tests/test_configs_gpu.py -k "not config5" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn1w_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/attn1w_tests.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/ab_1w_v2.log
for i in 1 2 3; do
for k in 1w 2w; do
  CP25_ATTN_KERNEL=$k timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 > /tmp/o.txt 2>&1 || exit 1
  echo "$k $(grep '^{' /tmp/o.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms"],2), round(d["tflops"]), d["check_rel_l2"])')" | tee -a gpurun_out/ab_1w_v2.log
done
done
