#!/bin/bash
# round 6 lab: same-box A/B of attn_fwd_w64 lab variants (tools/lab/w64/libcp25_<v>.so) against attn_fwd_m16 at the
# metric shape (the DiT's fused form), one process per variant, m16 and w64 alternating inside each
set -o pipefail
OUT=gpurun_out/${OUT:-r6c}
mkdir -p $OUT
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
for v in "$@"; do
  timeout -k 10 150 python -u tools/bench_attn.py --fused --bounded --prescaled --qnorm --iters 4 --ab 3 \
    --lib tools/lab/w64/libcp25_$v.so > $OUT/iso_$v.json 2> $OUT/iso_$v.err || exit $?
  python -c "import json; d=json.load(open('$OUT/iso_$v.json')); print('$v', d['ab_ms'], round(d['check_rel_l2'], 5))"
done
