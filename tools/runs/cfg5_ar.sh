# config 5 (action-conditioned AR, 480x640, 512 frames): fp8 GEMMs with / without fp8 Q K^T, bf16; same box
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/cfg5
timeout -k 10 300 python tools/bench_action_ar.py --linear-precision fp8 --attention-precision fp8 > gpurun_out/cfg5/fp8_fp8attn.json 2> gpurun_out/cfg5/e1.err && \
timeout -k 10 300 python tools/bench_action_ar.py --linear-precision fp8 > gpurun_out/cfg5/fp8.json 2> gpurun_out/cfg5/e2.err && \
timeout -k 10 300 python tools/bench_action_ar.py > gpurun_out/cfg5/bf16.json 2> gpurun_out/cfg5/e3.err
rc=$?
tail -n1 gpurun_out/cfg5/*.json
exit $rc
