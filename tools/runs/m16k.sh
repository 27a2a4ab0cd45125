# m16 MFMA-phase anatomy: V from the qkv layout (two transposed reads per operand) vs V^T tiles (one ds_read_b128)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/m16k
rm -f gpurun_out/m16k/*.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_probe.py --L 109120 --prescaled --t0 600 --lib tools/lab/libattn_probe_base.so >> gpurun_out/m16k/probe.log 2>&1 || exit 1
  timeout -k 10 120 python tools/attn_probe.py --L 109120 --prescaled --vt --t0 600 --lib tools/lab/libattn_probe_base.so >> gpurun_out/m16k/probe.log 2>&1 || exit 1
done
grep '^{' gpurun_out/m16k/probe.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(round(d['ms'],1), 'A', d['A'], 'B', d['B'])"
