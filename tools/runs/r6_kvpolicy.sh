#!/bin/bash
# round 6: cache policy of the self-attention's K / V LDS-DMA (tools/lab/attn_variant.py kv_*): same-process A/B at the
# metric launch (B 2, H 16, L 109 120, the DiT's fused q-norm form), product library vs the variants, bit-identity
set -o pipefail
O=gpurun_out/${OUT:-r6_kvpolicy}
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
L=tools/lab
timeout -k 10 400 python -u tools/bench_attn.py --fused --bounded --prescaled --qnorm --iters 4 --ab 6 \
  --ab-libs ${LIBS:-$L/libcp25_none.so,$L/libcp25_kv_sc1.so,$L/libcp25_kv_nt.so,$L/libcp25_kv_sc0sc1.so} > $O/ab_unit.json 2> $O/ab_unit.err || { tail -5 $O/ab_unit.err; exit 1; }
cat $O/ab_unit.json
