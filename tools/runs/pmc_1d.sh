set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_1d gpurun_out/pmc_2w
CP25_ATTN_KERNEL=1d timeout -k 10 400 bash tools/pmc_attn.sh gpurun_out/pmc_1d && python3 tools/pmc_summary.py gpurun_out/pmc_1d > gpurun_out/pmc_1d/SUMMARY.json && cat gpurun_out/pmc_1d/SUMMARY.json
