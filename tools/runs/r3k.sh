#!/bin/bash
# round 3k: the 8-wave halo conv as default (conv + VAE tests, PMC at the 96-channel shape); config 5's M (9 600 rows
# = 4 800 tokens x CFG 2): own GEMMs vs the library, bf16 and fp8; the config-5 action AR loop (512 frames at 480x640)
# with own vs library block GEMMs, bf16 and fp8
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3k
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_conv_halo_gpu.py \
  tests/test_vae_gpu.py -k "not metric_geometry" > gpurun_out/r3k/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3k/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r3k/tests.log | tail -1
export CONV_SHAPE=0
bash tools/pmc_passes.sh gpurun_out/r3k/pmc_conv python3 tools/bench_conv.py || exit 1
python3 tools/pmc_summary.py gpurun_out/r3k/pmc_conv --kernel "conv3x3_halo_kernel<3, 128, 8>" --name "halo conv (8 waves) 96->96 704x1280 Tout 4" \
  --flop 1793819934720 --algo-bytes 1730648064 > gpurun_out/r3k/pmc_conv.json && cat gpurun_out/r3k/pmc_conv.json
unset CONV_SHAPE
timeout -k 10 200 python tools/bench_gemm.py --M 9600 --plain --rounds 3 > gpurun_out/r3k/gemm_m9600_bf16.log 2>&1 || { tail gpurun_out/r3k/gemm_m9600_bf16.log; exit 1; }
timeout -k 10 200 python tools/bench_gemm.py --M 9600 --plain --rounds 3 --fp8 > gpurun_out/r3k/gemm_m9600_fp8.log 2>&1 || { tail gpurun_out/r3k/gemm_m9600_fp8.log; exit 1; }
cut -c1-260 gpurun_out/r3k/gemm_m9600_bf16.log gpurun_out/r3k/gemm_m9600_fp8.log | grep "{"
for lp in bf16 fp8; do
  for g in own lib; do
    timeout -k 10 300 python tools/bench_action_ar.py --linear-precision $lp --block-gemm $g > gpurun_out/r3k/ar_${lp}_$g.json 2> gpurun_out/r3k/ar_${lp}_$g.err || { tail gpurun_out/r3k/ar_${lp}_$g.err; exit 1; }
    cat gpurun_out/r3k/ar_${lp}_$g.json
  done
done
