set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for p in bf16 fp8; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --linear-precision $p > gpurun_out/benchfull_$p.log 2> gpurun_out/benchfull_$p.err || exit 1
  python3 -c "import json; j=json.loads(open('gpurun_out/benchfull_$p.log').read().strip().splitlines()[-1]); print('$p', j['value'], j['ms_per_step'], j['roofline']['avg_launch_ms'])"
done
