set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/sim_cp_rank.py --model 14B/pre-trained --cp 1 8 --iters 2 > gpurun_out/sim14.log 2>&1
rc=$?; grep '{' gpurun_out/sim14.log; exit $rc
