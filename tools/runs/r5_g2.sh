#!/bin/bash
# round 5: rehearsal of the self-launched multi-rank bench flow on one GPU (2 gloo ranks sharing cuda:0), and the
# library fp32 GEMMs left on the evaluation path timed (the final linear, the t-embedding / AdaLN linears)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r5g2
mkdir -p $O
timeout -k 10 900 python bench.py --gpus 2 --backend gloo --share-device --steps 2 --warmup 1 --num-steps 3 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -30 $O/bench_gloo2.err; exit 1; }
tail -1 $O/bench_gloo2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['value_method'], json.dumps(d.get('context_parallel'))[:400])"
timeout -k 10 120 python3 - <<'PY'
import torch, torch.nn.functional as F
dev = torch.device("cuda:0")
def t(fn, it=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / it
x = torch.randn(218240, 2048, device=dev); w = torch.randn(64, 2048, device=dev)
ms = t(lambda: F.linear(x, w))
print("final linear fp32 [218240,2048]x[64,2048]^T", round(ms, 3), "ms", round(2*218240*64*2048/ms/1e9, 1), "TF/s",
      "tf32 allowed:", torch.backends.cuda.matmul.allow_tf32)
ref = (x.double() @ w.double().t())
print("rel err vs fp64", ((F.linear(x, w).double() - ref).norm() / ref.norm()).item())
for (M, N, K) in ((62, 2048, 2048), (62, 6144, 2048), (62, 21504, 2048)):
    a = torch.randn(M, K, device=dev); b = torch.randn(N, K, device=dev)
    print("fp32", M, N, K, round(t(lambda: F.linear(a, b)), 4), "ms")
PY
