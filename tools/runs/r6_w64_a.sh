#!/bin/bash
# round 6: first GPU run of attn_fwd_w64 -- bit-identity vs attn_fwd_m16, then a same-process A/B at the metric shape
set -o pipefail
mkdir -p gpurun_out/${OUT:-r6a}
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 600 python -u -m pytest tests/test_attn_w64_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${OUT:-r6a}/tests_w64.log 2>&1
rc=$?
tail -5 gpurun_out/${OUT:-r6a}/tests_w64.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/bench_attn.py --fused --bounded --prescaled --qnorm --iters 5 --ab 4 > gpurun_out/${OUT:-r6a}/ab_unit.json 2> gpurun_out/${OUT:-r6a}/ab_unit.err || exit $?
cat gpurun_out/${OUT:-r6a}/ab_unit.json
timeout -k 10 300 python -u tools/bench_attn.py --fused --bounded --prescaled --qnorm --wrange 0.5,3 --iters 5 --ab 4 > gpurun_out/${OUT:-r6a}/ab_trained.json 2> gpurun_out/${OUT:-r6a}/ab_trained.err || exit $?
cat gpurun_out/${OUT:-r6a}/ab_trained.json
