#!/bin/bash
# round 6: descriptor-ABI + GELU-epilogue tests, the GELU table vs VALU A/B, and the LDS bank-conflict PMC of both
set -o pipefail
O=gpurun_out/${OUT:-r6_gelu}
mkdir -p $O
export PYTHONPATH=$PWD/cosmos-predict2.5_amd
timeout -k 10 600 python -u -m pytest tests/test_tensor_abi_gpu.py tests/test_gemm_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/lab/gelu/ab_gelu.py > $O/ab_gelu.json 2> $O/ab_gelu.err || { tail -20 $O/ab_gelu.err; exit 1; }
cat $O/ab_gelu.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for f in table valu; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES -d $O/pmc_$f -o pmc -- python3 tools/lab/gelu/ab_gelu.py --only $f > $O/pmc_$f.log 2>&1 || { tail -20 $O/pmc_$f.log; exit 1; }
done
echo pmc done
