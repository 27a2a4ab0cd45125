set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r2.log 2> gpurun_out/bench_r2.err
rc=$?; tail -c 2500 gpurun_out/bench_r2.log; exit $rc
