set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 60 python tools/bench_attn.py --L 109120 --iters 3 > gpurun_out/ba.log 2>&1 && \
timeout -k 10 60 python tools/bench_attn.py --L 13640 --Lk 109120 --split 1 --iters 5 >> gpurun_out/ba.log 2>&1 && \
timeout -k 10 60 python tools/bench_attn.py --L 13640 --Lk 109120 --iters 5 >> gpurun_out/ba.log 2>&1 && \
timeout -k 10 60 python tools/bench_attn.py --L 13640 --Lk 109120 --H 4 --split 1 --iters 5 >> gpurun_out/ba.log 2>&1 && \
timeout -k 10 60 python tools/bench_attn.py --L 13640 --Lk 109120 --H 4 --iters 5 >> gpurun_out/ba.log 2>&1 && \
timeout -k 10 60 python tools/bench_attn.py --L 27280 --Lk 109120 --H 4 --iters 5 >> gpurun_out/ba.log 2>&1 && \
timeout -k 10 60 python tools/bench_attn.py --L 54560 --Lk 109120 --H 4 --iters 5 >> gpurun_out/ba.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; cat gpurun_out/ba.log; exit $rc
