set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 60 python tools/bench_attn.py --L 109120 --iters 3 --bounded 2>/dev/null | grep '{'
