set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 100 python tools/sim_cp_rank.py --cp 2 --gather expand --blocks 2 --iters 1 > gpurun_out/sim_dbg.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/sim_dbg.log | tail -40; exit $rc
