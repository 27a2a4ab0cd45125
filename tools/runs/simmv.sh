set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python tools/sim_cp_rank.py --model 2B/auto/multiview --geometry 105,27,48 --views 7 --cp 1 8 --iters 2 > gpurun_out/simmv.log 2>&1
rc=$?; grep '{' gpurun_out/simmv.log; tail -3 gpurun_out/simmv.log; exit $rc
