set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/qrow_ab.log
for r in 1 2; do
  timeout -k 10 100 python tools/bench_quant_fp8.py 2>/dev/null | grep '"gelu": true' >> gpurun_out/qrow_ab.log || exit 1
  for v in w4n4 w8n2 w4n4b16 w8n2b16; do
    timeout -k 10 100 python tools/bench_quant_fp8.py --lib tools/lab/libcp25_q$v.so 2>/dev/null | grep '"gelu": true' >> gpurun_out/qrow_ab.log || exit 1
  done
done
python3 -c "
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/qrow_ab.log'):
    j = json.loads(l); d[(j['lib'], j['M'])].append(round(j['ms'], 4))
for k, v in sorted(d.items()): print(k, v)
"
