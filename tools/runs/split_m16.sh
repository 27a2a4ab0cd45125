# key-range split choice for the 16x16x32 kernel at the CP lanes' shapes (B 1 per lane, H 16)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/split
rm -f gpurun_out/split/*.log
for shape in "13640 109120" "27280 109120" "17010 136080"; do
  set -- $shape
  for s in 0 1 2 3 4; do
    timeout -k 10 120 python tools/bench_attn.py --bounded --prescaled --iters 6 --B 1 --L $1 --Lk $2 --split $s >> gpurun_out/split/split.log 2>&1 || exit 1
  done
done
python3 -c "
import json
for l in open('gpurun_out/split/split.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['Lq'], d['Lk'], d['split'], round(d['ms'],3))"
