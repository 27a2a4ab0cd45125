set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 180 python tools/bench_block_linear.py > gpurun_out/block_linear.log 2> gpurun_out/block_linear.err
rc=$?; cat gpurun_out/block_linear.log; [ $rc = 0 ] || exit $rc
for p in bf16 fp8; do
  timeout -k 10 300 python bench.py --num-steps 4 --no-cpu-baseline --linear-precision $p > gpurun_out/bench4_$p.log 2> gpurun_out/bench4_$p.err || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/bench4_$p.log').read().strip().splitlines()[-1]); print('$p', j['ms_per_step'], j['phases_last_step_s'], j['roofline']['avg_launch_ms'])"
done
