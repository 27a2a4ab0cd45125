#!/bin/bash
# round 3i: attention tests (cross-only 16-B stores), PMC passes of the self-attention, the cross-attention and the
# 96-channel halo conv at their bench shapes
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3i
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -s tests/test_attn_m16_gpu.py \
  tests/test_attention_gpu.py > gpurun_out/r3i/tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/r3i/tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/r3i/tests.log | tail -1
bash tools/pmc_passes.sh gpurun_out/r3i/pmc_self python3 tools/bench_attn.py --iters 1 --bounded --fused --prescaled || exit 1
python3 tools/pmc_summary.py gpurun_out/r3i/pmc_self > gpurun_out/r3i/pmc_self.json && cat gpurun_out/r3i/pmc_self.json
bash tools/pmc_passes.sh gpurun_out/r3i/pmc_cross python3 tools/bench_attn.py --iters 3 --bounded --prescaled --Lk 512 || exit 1
python3 tools/pmc_summary.py gpurun_out/r3i/pmc_cross --kernel "attn_fwd_m16<1" --name "cross-attention B=2 H=16 Lq=109120 Lk=512" \
  --flop 915364904960 --algo-bytes 1796210688 > gpurun_out/r3i/pmc_cross.json && cat gpurun_out/r3i/pmc_cross.json
export CONV_SHAPE=0
bash tools/pmc_passes.sh gpurun_out/r3i/pmc_conv python3 tools/bench_conv.py || exit 1
python3 tools/pmc_summary.py gpurun_out/r3i/pmc_conv --kernel "conv3x3_halo_kernel<3, 128>" --name "halo conv 96->96 704x1280 Tout 4" \
  --flop 1793819934720 --algo-bytes 1730648064 > gpurun_out/r3i/pmc_conv.json && cat gpurun_out/r3i/pmc_conv.json
