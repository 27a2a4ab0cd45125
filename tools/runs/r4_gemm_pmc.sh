#!/bin/bash
# round 4: PMC passes of the own GEMM vs hipBLASLt at the MLP1 and QKV shapes (clock, MFMA busy, wave split,
# LDS conflicts, HBM bytes)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r4gp
mkdir -p $O
for s in mlp1 qkv; do
  bash tools/pmc_passes.sh $O/$s python3 tools/bench_gemm.py --plain --rounds 1 --shapes $s || exit 1
done
M=218240
python3 tools/pmc_summary.py $O/mlp1 --kernel gemm_nt_8ph --name "own mlp1" --flop $((2*M*8192*2048)) --algo-bytes $((2*(M*2048+8192*2048+M*8192))) > $O/own_mlp1.json
python3 tools/pmc_summary.py $O/mlp1 --kernel Cijk --name "hipblaslt mlp1" --flop $((2*M*8192*2048)) --algo-bytes $((2*(M*2048+8192*2048+M*8192))) > $O/lib_mlp1.json
python3 tools/pmc_summary.py $O/qkv --kernel gemm_nt_8ph --name "own qkv" --flop $((2*M*6144*2048)) --algo-bytes $((2*(M*2048+6144*2048+M*6144))) > $O/own_qkv.json
python3 tools/pmc_summary.py $O/qkv --kernel Cijk --name "hipblaslt qkv" --flop $((2*M*6144*2048)) --algo-bytes $((2*(M*2048+6144*2048+M*6144))) > $O/lib_qkv.json
cat $O/*.json
