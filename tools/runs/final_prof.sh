set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc_attn.sh gpurun_out/pmc_r1d && \
python tools/pmc_summary.py gpurun_out/pmc_r1d > gpurun_out/pmc_r1d/SUMMARY.json && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1d -o run -- python bench.py > gpurun_out/bench_r1d.log 2> gpurun_out/bench_r1d.err
rc=$?; cat gpurun_out/pmc_r1d/SUMMARY.json; tail -1 gpurun_out/bench_r1d.log | cut -c1-400; exit $rc
