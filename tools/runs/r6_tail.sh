#!/bin/bash
# round 6: GEMM tail row slices -- the GEMM / CP suites, the same-process A/B against the whole-tile plan, and the
# CP = 8 rank simulation with the gather hidden (2B, 14B)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-r6_tail}
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_qkv_gpu.py tests/test_gemm_hnorm_gpu.py tests/test_fp8_gpu.py tests/test_configs_net_gpu.py tests/test_cp_gpu.py tests/test_op_table_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | tail -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
grep -E "CP=8 rank" $O/tests.log | head -4
timeout -k 10 300 python -u tools/lab/gemm_tail/ab_tail.py > $O/ab_tail.jsonl 2> $O/ab_tail.err || { tail -20 $O/ab_tail.err; exit 1; }
python3 -c "
import json
for l in open('$O/ab_tail.jsonl'):
    d = json.loads(l); print(d['M'], d['gemm'], d['tiles'], d['bit_identical'], d['slices_min'], d['base_min'], round(d['speedup'], 4))"
timeout -k 10 900 python tools/sim_cp_rank.py --cp 1 8 --iters 2 --gather none > $O/sim2b_none.log 2> $O/sim2b_none.err || { tail -20 $O/sim2b_none.err; exit 1; }
timeout -k 10 900 python tools/sim_cp_rank.py --model 14B/pre-trained --cp 1 8 --iters 1 --gather none > $O/sim14_none.log 2> $O/sim14_none.err || { tail -20 $O/sim14_none.err; exit 1; }
for f in sim2b_none sim14_none; do echo $f; grep "^{" $O/$f.log | python3 -c "
import json, sys
rows = [json.loads(l) for l in sys.stdin]
base = [r for r in rows if r['cp'] == 1][0]['forward_s']
for r in rows:
    print(r['cp'], round(r['forward_s'], 4), 'eff', round(base / r['cp'] / r['forward_s'], 4))"
done
