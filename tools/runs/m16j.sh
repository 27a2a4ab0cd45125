# m16 MFMA-phase anatomy: phase start -> first operand pair, the P.V half, the Q K^T half (s_memtime stamps)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16j
rm -f gpurun_out/m16j/*.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_probe.py --L 109120 --prescaled --t0 600 --lib tools/lab/libattn_probe_base.so >> gpurun_out/m16j/probe.log 2>&1 || exit 1
done
grep '^{' gpurun_out/m16j/probe.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(round(d['ms'],1), 'A', d['A'], 'B', d['B'])"
