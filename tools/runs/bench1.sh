set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 700 python bench.py 2> gpurun_out/bench.err | tee gpurun_out/bench.log
