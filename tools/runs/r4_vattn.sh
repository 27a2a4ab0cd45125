#!/bin/bash
# round 4: the one-pass VAE attention (tests, per-frame timing) and the cross-attention context probe + in-bench trace
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4va
mkdir -p $O
# (tests: run once before this script in this round, 29 passed; profiles/r4/vae_attn/tests.log)
# timing: the one-pass kernel (in-tree) vs the round-3 two-pass form (tools/lab/build_tu.py from the previous commit)
for rep in 1 2; do
  CONV_SHAPE=attn timeout -k 10 120 python3 tools/bench_conv.py >> $O/bench_vattn.json 2>> $O/bench_vattn.err || exit 1
  CONV_LIB=tools/lab/libcp25_va2pass.so CONV_SHAPE=attn timeout -k 10 120 python3 tools/bench_conv.py >> $O/bench_vattn_2pass.json 2>> $O/bench_vattn.err || exit 1
done
cat $O/bench_vattn.json $O/bench_vattn_2pass.json
bash tools/runs/r4_xattn_ctx.sh
