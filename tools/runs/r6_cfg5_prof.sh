#!/bin/bash
# round 6: config 5 (action AR, L = 4 800 per chunk) under rocprofv3 --kernel-trace: is its evaluation loop
# launch-bound? (busy fraction of the device between the first and last self-attention launch)
set -o pipefail
export PYTHONUNBUFFERED=1
O=$PWD/gpurun_out/r6_cfg5prof
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/bench_action_ar.py --frames 61 ${ARGS:-} > $O/ar.json 2> $O/ar.err || { tail -20 $O/ar.err; exit 1; }
cd $R
tail -n1 $O/ar.json | cut -c1-300
python3 tools/trace_gaps_db.py $(find $O/prof -name "*.db" | head -1) --json $O/gaps.json | head -12
