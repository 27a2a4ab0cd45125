#!/bin/bash
# round 4: GEMM tile seam with the next tile's K-tile 0 issued before the C staging (halves through buffer 1): tests, then
# a same-box A/B against the round-3 seam (tools/lab/libcp25_gprek0.so), bf16 and fp8, at the bench's M = 218 240
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_op_table_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for pass in 1 2; do
  for lib in tools/lab/libcp25_gprek0.so cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so; do
    timeout -k 10 200 python tools/bench_gemm.py --rounds 2 --lib $lib 2>$O/err.log >> $O/bf16_ab.log || { tail $O/err.log; exit 1; }
    timeout -k 10 200 python tools/bench_gemm.py --rounds 2 --fp8 --lib $lib 2>$O/err.log >> $O/fp8_ab.log || { tail $O/err.log; exit 1; }
  done
done
for f in bf16 fp8; do echo "== $f"; python3 -c "
import json, collections
r = collections.defaultdict(list); lib = collections.defaultdict(list)
for l in open('$O/${f}_ab.log'):
    if not l.startswith('{'): continue
    d = json.loads(l); r[(d['gemm'], d['lib'])] += d['own_ms']; lib[d['gemm']] += d.get('hipblaslt_ms', d.get('scaled_mm_ms', []))
fused = collections.defaultdict(list)
for l in open('$O/${f}_ab.log'):
    if not l.startswith('{'): continue
    d = json.loads(l)
    for k in ('own_gelu_fused_ms', 'own_residual_fused_plus_ln_mod_ms'):
        if k in d: fused[(d['gemm'], d['lib'], k)].append(d[k])
for (g, l), v in sorted(r.items()): print(g, l, 'own min', round(min(v), 4), 'library min', round(min(lib[g]), 4))
for (g, l, k), v in sorted(fused.items()): print(g, l, k, round(min(v), 4))"; done
