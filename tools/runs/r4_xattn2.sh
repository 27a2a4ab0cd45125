#!/bin/bash
# round 4: persistent cross-attention O staging, 264-B rows read by b64 pairs: tests, A/B vs round 3, one PMC pass
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4x2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_xattn_persistent_gpu.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for pass in 1 2 3; do
  for lib in tools/lab/libcp25_prexo.so cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so; do
    timeout -k 10 120 python tools/bench_xattn.py --forms 1 --rounds 2 --lib $lib 2>$O/err.log >> $O/xattn_ab.log || { tail $O/err.log; exit 1; }
  done
done
python3 -c "
import json, collections
r = collections.defaultdict(list)
for l in open('$O/xattn_ab.log'):
    d = json.loads(l); r[d['lib']].append(d['ms'])
for k, v in r.items(): print('xattn', k, [round(x, 4) for x in v], 'min', min(v))"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace --output-format csv \
  -d $O/pmc -o p -- python tools/bench_xattn.py --forms 1 --rounds 1 --iters 3 > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
f=$(find $O/pmc -name "*counter_collection.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
s = collections.defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    if "attn_fwd_m16" in row.get("Kernel_Name", ""):
        s[row["Counter_Name"]].append(float(row["Counter_Value"]))
print({k: sum(v) for k, v in s.items()})
PY
