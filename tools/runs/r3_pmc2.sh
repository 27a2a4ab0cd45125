#!/bin/bash
# round 3 (session 2): PMC passes of the nop-free self-attention, the persistent cross-attention and the 16x32-tile
# halo conv at their bench shapes
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3pmc
bash tools/pmc_passes.sh gpurun_out/r3pmc/pmc_self python3 tools/bench_attn.py --iters 1 --bounded --fused --prescaled || exit 1
python3 tools/pmc_summary.py gpurun_out/r3pmc/pmc_self > gpurun_out/r3pmc/pmc_self.json && cat gpurun_out/r3pmc/pmc_self.json
bash tools/pmc_passes.sh gpurun_out/r3pmc/pmc_cross python3 tools/bench_attn.py --iters 3 --bounded --prescaled --Lk 512 || exit 1
python3 tools/pmc_summary.py gpurun_out/r3pmc/pmc_cross --kernel "attn_fwd_m16<1" --name "cross-attention (persistent) B=2 H=16 Lq=109120 Lk=512" \
  --flop 915364904960 --algo-bytes 1796210688 > gpurun_out/r3pmc/pmc_cross.json && cat gpurun_out/r3pmc/pmc_cross.json
export CONV_SHAPE=0
bash tools/pmc_passes.sh gpurun_out/r3pmc/pmc_conv python3 tools/bench_conv.py || exit 1
python3 tools/pmc_summary.py gpurun_out/r3pmc/pmc_conv --kernel "conv3x3_halo_kernel<3, 32" --name "halo conv (16x32 tiles, 8 waves) 96->96 704x1280 Tout 4" \
  --flop 1793819934720 --algo-bytes 1730648064 > gpurun_out/r3pmc/pmc_conv.json && cat gpurun_out/r3pmc/pmc_conv.json
