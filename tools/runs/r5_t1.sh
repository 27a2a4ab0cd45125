#!/bin/bash
# round 5: attention / parity GPU tests on the changed tree (V by DMA in the zero-shift form, flash-class oracle rows)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5t1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_attn_m16_gpu.py tests/test_attn_qnorm_gpu.py tests/test_attention_gpu.py tests/test_attn_gated_gpu.py tests/test_attn_op_gpu.py tests/test_xattn_persistent_gpu.py tests/test_patch_embed_gpu.py tests/test_op_table_gpu.py tests/test_parity_depth_gpu.py -x -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|hip-ref|hip-vs|exact_q=" $O/tests.log | tail -40
exit $rc
