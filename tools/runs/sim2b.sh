set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/sim_cp_rank.py --cp 1 2 4 8 --iters 2 > gpurun_out/sim2b.log 2>&1
rc=$?; grep '{' gpurun_out/sim2b.log; exit $rc
