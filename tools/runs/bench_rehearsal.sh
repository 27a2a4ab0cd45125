set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --share-device --frames 9 --resolution 256,320 --num-steps 2 --no-cpu-baseline > gpurun_out/rehearsal2.log 2> gpurun_out/rehearsal2.err && \
timeout -k 10 300 python bench.py --frames 9 --resolution 256,320 --num-steps 2 --no-cpu-baseline > gpurun_out/rehearsal1.log 2> gpurun_out/rehearsal1.err
rc=$?; tail -1 gpurun_out/rehearsal2.log | cut -c1-300; tail -1 gpurun_out/rehearsal1.log | cut -c1-300; tail -5 gpurun_out/rehearsal2.err; exit $rc
