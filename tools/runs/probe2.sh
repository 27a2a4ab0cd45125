set -o pipefail
export PYTHONUNBUFFERED=1
: > gpurun_out/probe.log
for l in libattn_probe libattn_probe_head; do
  timeout -k 10 120 python tools/attn_probe.py --L 109120 --t0 800 --bounded --lib tools/lab/$l.so 2>&1 | grep '{' >> gpurun_out/probe.log || exit 1
done
cat gpurun_out/probe.log
