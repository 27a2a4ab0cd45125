# m16: row-sum MFMAs in the softmax phase vs in the MFMA phase (probe + metric-shape A/B)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16i
rm -f gpurun_out/m16i/*.log
for n in base lsm; do
  timeout -k 10 120 python tools/attn_probe.py --L 109120 --prescaled --t0 600 --lib tools/lab/libattn_probe_$n.so >> gpurun_out/m16i/probe.log 2>&1 || exit 1
done
grep '^{' gpurun_out/m16i/probe.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(round(d['ms'],1), 'A', d['A'], 'B', d['B'])"
for i in 1 2; do
  for n in base lsm; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 --lib tools/lab/libcp25_$n.so >> gpurun_out/m16i/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*\|"check_rel_l2": [0-9.e-]*' gpurun_out/m16i/ab.log | paste - - -
