# per-rank compute of CP = 1/2/4/8 at the metric shape with the 16x16x32 attention (collectives replaced by local copies)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/sim
timeout -k 10 500 python tools/sim_cp_rank.py --cp 1 2 4 8 --iters 2 > gpurun_out/sim/sim2b_m16.log 2>&1
rc=$?; grep '^{' gpurun_out/sim/sim2b_m16.log | cut -c1-300; exit $rc
