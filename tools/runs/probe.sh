set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/attn_probe.py --L 109120 --t0 800 > gpurun_out/probe.log 2>&1
rc=$?; grep '{' gpurun_out/probe.log; exit $rc
