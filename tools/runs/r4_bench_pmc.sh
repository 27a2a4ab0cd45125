#!/bin/bash
# round 4: one PMC pass (clock, MFMA busy, wave split) over a one-evaluation bench: the cross-attention, the
# self-attention and the GEMMs as they run inside the DiT (their last dispatch), for comparison with the standalone runs
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
O=gpurun_out/r4bp
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O -o p3 -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-whole-video > $O/bench.log 2>&1 || exit 1
M=218240
python3 tools/pmc_summary.py $O --kernel "attn_fwd_m16<1, true, 1, true" --name "cross-attention in bench" --flop $((4*2*16*109120*512*128)) --algo-bytes $((4*M*2048)) > $O/xattn.json
python3 tools/pmc_summary.py $O --kernel "attn_fwd_m16<0, true, 1, false" --name "self-attention in bench" > $O/self.json
python3 tools/pmc_summary.py $O --kernel "gemm_nt_8ph<1, 2>" --name "MLP1+GELU in bench" --flop $((2*M*8192*2048)) --algo-bytes $((2*(M*2048+8192*2048+M*8192))) > $O/mlp1.json
python3 tools/pmc_summary.py $O --kernel "gemm_nt_8ph<0, 2>" --name "plain GEMM (last: cross-q) in bench" --flop $((2*M*2048*2048)) --algo-bytes $((2*(M*2048+2048*2048+M*2048))) > $O/plain.json
python3 tools/pmc_summary.py $O --kernel "head_rmsnorm_rope" --name "head rmsnorm in bench" --flop 1 --algo-bytes $((4*M*2048)) > $O/norm.json
cat $O/*.json
