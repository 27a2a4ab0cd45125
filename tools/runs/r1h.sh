set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
bash tools/pmc_attn.sh gpurun_out/pmc_r1e && \
python tools/pmc_summary.py gpurun_out/pmc_r1e > gpurun_out/pmc_r1e/SUMMARY.json && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1e -o run -- python bench.py > gpurun_out/bench_r1e.log 2> gpurun_out/bench_r1e.err
rc=$?; cat gpurun_out/pmc_r1e/SUMMARY.json; tail -1 gpurun_out/bench_r1e.log | cut -c1-600; exit $rc
