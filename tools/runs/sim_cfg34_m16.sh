# configs 3 (14B, CP 8) and 4 (7-view multiview, CP 8): per-rank compute with the 16x16x32 attention
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/sim
timeout -k 10 500 python tools/sim_cp_rank.py --model 14B/pre-trained --cp 1 8 --iters 2 > gpurun_out/sim/sim14_m16.log 2>&1 && \
timeout -k 10 500 python tools/sim_cp_rank.py --model 2B/auto/multiview --geometry 105,27,48 --views 7 --cp 1 8 --iters 2 > gpurun_out/sim/simmv_m16.log 2>&1
rc=$?; grep -h '^{' gpurun_out/sim/sim14_m16.log gpurun_out/sim/simmv_m16.log | cut -c1-260; exit $rc
