"""Lab: per-wave cycle split of attn_fwd_w64 (a -DCP25_ATTN_PROBE -DCP25_W64_PROBE build, tools/lab/w64): loop cycles
per tile, the end-of-iteration vmcnt(0) wait, the barrier, and the in-kernel clock, at the metric launch shape."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, "cosmos-predict2.5_amd")
from cosmos_predict2 import _native as N  # noqa: E402

N._LIB_PATH = sys.argv[1]
dev = torch.device("cuda:0")
L, B, H = 109120, 2, 16
C = 128 ** -0.5 * 1.4426950408889634
g = torch.Generator(device=dev).manual_seed(3)
buf = torch.randn(L, B, 3 * H * 128, device=dev, generator=g).to(torch.bfloat16)
q, k, v = (buf[:, :, i * H * 128:(i + 1) * H * 128].view(L, B, H, 128).transpose(0, 1) for i in range(3))
w = torch.ones(128, device=dev)
k.copy_((k.float() * torch.rsqrt(k.float().pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16))
ang = torch.rand(L, 64, device=dev) * 50.0
qn = dict(weight=w.to(torch.bfloat16), cos=torch.cos(ang).contiguous(), sin=torch.sin(ang).contiguous(), out_scale=C)
wb = 128 ** 0.5 * 1.02
nb = (wb * C, wb)
N.attn_self_select(1)
for _ in range(6):  # warm the clock
    o = N.attn_fwd(q, k, v, prescaled=True, norm_bounds=nb, q_norm=qn)
torch.cuda.synchronize()
lib = N.load_library()
lib.cp25_attn_probe_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
nwg = int(sys.argv[2]) if len(sys.argv) > 2 else 256
pb = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device=dev)
lib.cp25_attn_probe_set(ctypes.c_void_p(pb.data_ptr()), 0, nwg)
o = N.attn_fwd(q, k, v, prescaled=True, norm_bounds=nb, q_norm=qn, n_split=1)
torch.cuda.synchronize()
lib.cp25_attn_probe_set(None, 0, 0)
x = pb.view(nwg, 4, 8).double().cpu()
T = x[..., 3]
per = lambda i: (x[..., i] / T).median().item()
print(json.dumps({"loop_cyc_per_tile": round(per(0), 1), "vmcnt_wait_per_tile": round(per(1), 1),
                  "barrier_per_tile": round(per(2), 1), "clock_ghz": round((x[..., 0] / x[..., 4]).median().item() / 10, 3),
                  "wait_p90": round(torch.quantile(x[..., 1] / T, 0.9).item(), 1), "tiles": T.median().item(),
                  "mfma_floor_per_tile": 136 * 16}))
