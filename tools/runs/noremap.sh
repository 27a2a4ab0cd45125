# m16: XCD-remapped tile order vs dispatch order (all XCDs on one (b, h) at a time: K/V working set in the MALL)
set -o pipefail
export PYTHONUNBUFFERED=1
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$root"
mkdir -p gpurun_out/noremap
rm -f gpurun_out/noremap/*.log
for i in 1 2; do
  for n in base noremap; do
    timeout -k 10 120 python tools/bench_attn.py --fused --bounded --prescaled --iters 4 --lib tools/lab/libcp25_$n.so >> gpurun_out/noremap/ab.log 2>&1 || exit 1
  done
done
grep -o '"lib": "[^"]*"\|"ms": [0-9.]*\|"check_rel_l2": [0-9.e-]*' gpurun_out/noremap/ab.log | paste - - -
for n in base noremap; do
  mkdir -p gpurun_out/noremap/pmc_$n
  timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/noremap/pmc_$n -o p1 -- \
    python3 tools/bench_attn.py --L 109120 --B 2 --iters 1 --bounded --fused --prescaled --lib tools/lab/libcp25_$n.so > gpurun_out/noremap/pmc_$n/p1.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/noremap/pmc_$n | grep -E "hbm_read|duration" || true
done
