# m16: group B pre-issues its first MFMA-phase reads before the barrier (probe + metric-shape A/B)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16h
rm -f gpurun_out/m16h/*.log
for n in base preb; do
  timeout -k 10 120 python tools/attn_probe.py --L 109120 --prescaled --t0 600 --lib tools/lab/libattn_probe_$n.so >> gpurun_out/m16h/probe.log 2>&1 || exit 1
done
grep '^{' gpurun_out/m16h/probe.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(round(d['ms'],1), 'A', d['A'], 'B', d['B'])"
for i in 1 2; do
  for n in base preb; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 --lib tools/lab/libcp25_$n.so >> gpurun_out/m16h/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*\|"check_rel_l2": [0-9.e-]*' gpurun_out/m16h/ab.log | paste - - -
