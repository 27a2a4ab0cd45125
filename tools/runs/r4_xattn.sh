#!/bin/bash
# round 4: swizzled O staging of the persistent cross-attention: tests, same-box A/B against the previous build
# (tools/lab/libcp25_prexo.so), then one PMC pass of the bank-conflict counters; plus the dot2 row-sum self-attention A/B
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_xattn_persistent_gpu.py tests/test_attn_m16_gpu.py -m gpu -x -v --timeout 300 \
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
for lib in tools/lab/libcp25_prexo.so cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so; do
  n=$(basename $lib .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace --output-format csv \
    -d $O/pmc_$n -o p -- python tools/bench_xattn.py --forms 1 --rounds 1 --iters 3 --lib $lib > $O/pmc_$n.log 2>&1 || { tail $O/pmc_$n.log; exit 1; }
done
for n in libcp25_prexo libcp25; do f=$(find $O/pmc_$n -name "*counter_collection.csv" | head -1); python3 - "$f" "$n" <<'PY'
import csv, sys, collections
s = collections.defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    if "attn_fwd_m16" in row.get("Kernel_Name", ""):
        s[row["Counter_Name"]].append(float(row["Counter_Value"]))
print(sys.argv[2], {k: sum(v) / max(1, len(set(range(len(v))))) for k, v in s.items()})
PY
done
LIBS="tools/lab/libcp25_rsdot2.so" bash tools/runs/r4_ab.sh rsdot2
