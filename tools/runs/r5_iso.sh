#!/bin/bash
# round 5: isolation builds of the self-attention loop with the s_memtime probe (WRONG results except probe / ahead3):
# which part of the MFMA phase's excess is the softmax VALU (noexp), the operand reads (noreads), or both; and the
# online form's cost split into cycles and clock: the same online kernel on unit-weight data (--force-online) vs on
# norm weights in [0.5, 3]
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5iso
mkdir -p $O
B="python3 tools/bench_attn.py --fused --bounded --prescaled --qnorm"
for lib in probe p_noexp p_noreads p_noexp_noreads p_ahead3; do
  for w in "1,1" "0.5,3"; do
    timeout -k 10 120 $B --wrange $w --iters 3 --lib tools/lab/libcp25_$lib.so --probe 800 --probe-dump $O/${lib}_${w/,/_}.npy >> $O/probe.jsonl 2>>$O/err.log || exit 1
  done
done
timeout -k 10 120 $B --wrange 1,1 --force-online --iters 3 --lib tools/lab/libcp25_probe.so --probe 800 >> $O/probe.jsonl 2>>$O/err.log || exit 1
for rep in 1 2; do
  for lib in cosmos-predict2.5_amd/cosmos_predict2/_lib/libcp25.so tools/lab/libcp25_ahead3.so; do
    for w in "1,1" "0.5,3"; do
      timeout -k 10 120 $B --wrange $w --iters 4 --lib $lib >> $O/ab.jsonl 2>>$O/err.log || exit 1
    done
  done
  timeout -k 10 120 $B --wrange 1,1 --force-online --iters 4 >> $O/ab.jsonl 2>>$O/err.log || exit 1
done
python3 - <<'PY'
import json
for l in open('gpurun_out/r5iso/probe.jsonl'):
    d = json.loads(l); p = d['probe']
    print(d['lib'], d['wrange'], 'forced-online' if d.get('force_online') else '', round(d['ms'], 2), {k: p.get(k) for k in ('period', 'A_mfma_span', 'B_mfma_span', 'A_softmax_span', 'B_softmax_span', 'X_release_after_last', 'Y_release_after_last', 'X_overrun_softmax_after_mfma', 'Y_overrun_softmax_after_mfma', 'clock_ghz', 'loop_cycles')})
for l in open('gpurun_out/r5iso/ab.jsonl'):
    d = json.loads(l); print(d['lib'], d['wrange'], 'forced-online' if d.get('force_online') else '', round(d['ms'], 2), d['check_rel_l2'])
PY
