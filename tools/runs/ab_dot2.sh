set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 120 python tools/check_attn_lib.py --lib tools/lab/libcp25_dot2.so > gpurun_out/dot2_check.log 2>&1
rc=$?; tail -n 4 gpurun_out/dot2_check.log; [ $rc = 0 ] || exit $rc
VARIANTS="base dot2" bash tools/runs/ab_attn.sh
