set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_attn_op_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn1w_tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/attn1w_tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  CP25_ATTN_KERNEL=2w timeout -k 10 120 python tools/bench_attn.py --fused --bounded --iters 5 >> gpurun_out/attn1w_ab.log 2>&1 || exit 1
  CP25_ATTN_KERNEL=1w timeout -k 10 120 python tools/bench_attn.py --fused --bounded --iters 5 >> gpurun_out/attn1w_ab.log 2>&1 || exit 1
done
CP25_ATTN_KERNEL=1w timeout -k 10 120 python tools/bench_attn.py --L 109120 --Lk 512 --bounded --iters 20 >> gpurun_out/attn1w_ab.log 2>&1
CP25_ATTN_KERNEL=2w timeout -k 10 120 python tools/bench_attn.py --L 109120 --Lk 512 --bounded --iters 20 >> gpurun_out/attn1w_ab.log 2>&1
cat gpurun_out/attn1w_ab.log | cut -c1-400
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/configs_gpu.log 2>&1
rc=$?; grep -E "rel-L2|passed|failed|Error" gpurun_out/configs_gpu.log | tail -8; exit $rc
