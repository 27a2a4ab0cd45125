set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_conv
bash tools/pmc_conv.sh gpurun_out/pmc_conv && python3 tools/pmc_conv_summary.py gpurun_out/pmc_conv > gpurun_out/pmc_conv/SUMMARY.json && cat gpurun_out/pmc_conv/SUMMARY.json
