set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for p in bf16 fp8; do
  timeout -k 10 400 python tools/bench_action_ar.py --linear-precision $p > gpurun_out/action_ar_$p.log 2> gpurun_out/action_ar_$p.err || { tail -5 gpurun_out/action_ar_$p.err; exit 1; }
  tail -n 1 gpurun_out/action_ar_$p.log
done
