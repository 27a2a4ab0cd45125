# config 5 (action-conditioned AR 512f, 480x640): fp8 GEMMs + whole-fp8 attention vs fp8 GEMMs alone, same box
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/cfg5
timeout -k 10 300 python tools/bench_action_ar.py --linear-precision fp8 --attention-precision fp8 > gpurun_out/cfg5/fp8_fp8attn_full.json 2> gpurun_out/cfg5/e1.err && \
timeout -k 10 300 python tools/bench_action_ar.py --linear-precision fp8 > gpurun_out/cfg5/fp8_b.json 2> gpurun_out/cfg5/e2.err
rc=$?
tail -n1 gpurun_out/cfg5/fp8_fp8attn_full.json gpurun_out/cfg5/fp8_b.json
exit $rc
