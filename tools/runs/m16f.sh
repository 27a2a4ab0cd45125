# m16 phase anatomy: default vs no softmax transcendental vs no MFMA-phase LDS reads (lab, wrong results)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16f
rm -f gpurun_out/m16f/*.log
for i in 1 2; do
for n in base noexp nolds; do
  timeout -k 10 120 python tools/attn_probe.py --L 109120 --prescaled --t0 600 --lib tools/lab/libattn_probe_$n.so >> gpurun_out/m16f/probe.log 2>&1 || exit 1
done
done
grep '^{' gpurun_out/m16f/probe.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(round(d['ms'],1), 'A', d['A'], 'B', d['B'])"
