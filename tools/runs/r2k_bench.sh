# the driver's bench command on the last tree (another box)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r2k
timeout -k 10 560 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2k/bench_driver_cmd.json 2> gpurun_out/r2k/bench_driver_cmd.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r2k/bench_driver_cmd.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config']['seconds_per_video'], d['roofline']['avg_launch_ms'], d['roofline']['achieved'], d['roofline']['frac'])"
