#!/bin/bash
# round 6: does P's magnitude move the self-attention's clock? (tools/lab/ab_shift_power.py)
set -o pipefail
O=gpurun_out/r6_shift
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 400 python -u tools/lab/ab_shift_power.py --rounds ${ROUNDS:-4} > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.json
