"""Phase anatomy of the self-attention kernel from in-kernel s_memtime stamps (lab build).

Build the instrumented library first (not part of the product):
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fno-honor-nans -DCP25_ATTN_PROBE -Iinclude \
        -shared -o tools/lab/libattn_probe.so cosmos-predict2.5_amd/csrc/attn_fwd.hip
usage: python tools/attn_probe.py [--L 32768] [--t0 200]
Prints, per wave group, the mean cycles of each phase and barrier wait over 32 tiles x 8 workgroups.
"""
import argparse
import ctypes
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=32768)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--t0", type=int, default=200)
    ap.add_argument("--bounded", action="store_true", help="RMS-normed q/k + cp25_attn_fwd_bounded (the DiT's form)")
    ap.add_argument("--prescaled", action="store_true", help="RMS-normed k, q * scale * log2(e) + cp25_attn_fwd_prescaled")
    ap.add_argument("--vt", action="store_true", help="with --prescaled: V as cp25_cast_v_bf16t tiles (_prescaled_vt)")
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "lab", "libattn_probe.so"))
    a = ap.parse_args()
    lib = ctypes.CDLL(a.lib)
    P = ctypes.c_void_p
    lib.cp25_attn_fwd.argtypes = [P, P, P, P] + [ctypes.c_int] * 5 + [P] * 4 + [ctypes.c_float, P]
    lib.cp25_attn_fwd.restype = ctypes.c_int
    lib.cp25_attn_fwd_bounded.argtypes = [P, P, P, P] + [ctypes.c_int] * 5 + [P] * 4 + [ctypes.c_float] * 3 + \
        [ctypes.c_int, P, ctypes.c_size_t, P]
    lib.cp25_attn_fwd_bounded.restype = ctypes.c_int
    lib.cp25_attn_fwd_prescaled.argtypes = [P, P, P, P] + [ctypes.c_int] * 5 + [P] * 4 + [ctypes.c_float] * 2 + \
        [ctypes.c_int, P, ctypes.c_size_t, P]
    lib.cp25_attn_fwd_prescaled.restype = ctypes.c_int
    lib.cp25_attn_fwd_prescaled_vt.argtypes = [P, P, P, P] + [ctypes.c_int] * 5 + [P] * 3 + [ctypes.c_float] * 2 + \
        [ctypes.c_int, P, ctypes.c_size_t, P]
    lib.cp25_attn_fwd_prescaled_vt.restype = ctypes.c_int
    lib.cp25_v_bf16t_bytes.argtypes = [ctypes.c_int] * 3
    lib.cp25_v_bf16t_bytes.restype = ctypes.c_int64
    lib.cp25_cast_v_bf16t.argtypes = [P, P] + [ctypes.c_int] * 4 + [P, P]
    lib.cp25_cast_v_bf16t.restype = ctypes.c_int
    lib.cp25_attn_probe_set.argtypes = [P, ctypes.c_int]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    q, k, v = (torch.randn(a.B, a.L, a.H, 128, device=dev, generator=g).to(torch.bfloat16) for _ in range(3))
    if a.bounded or a.prescaled:
        for t in (q, k):
            t.copy_((t.float() * torch.rsqrt(t.float().pow(2).mean(-1, keepdim=True) + 1e-6)).to(torch.bfloat16))
    c = 128 ** -0.5 * 1.4426950408889634
    if a.prescaled:
        q.copy_((q.float() * c).to(torch.bfloat16))
    o = torch.empty_like(q)
    probe = torch.zeros(8 * 8 * 32 * 8, dtype=torch.int64, device=dev)

    def strides(t):
        return (ctypes.c_int64 * 3)(t.stride(0), t.stride(1), t.stride(2))

    st = [strides(t) for t in (q, k, v, o)]
    stream = torch.cuda.current_stream().cuda_stream

    vt = None
    if a.vt:
        vt = torch.empty(lib.cp25_v_bf16t_bytes(a.B, a.H, a.L) // 2, dtype=torch.bfloat16, device=dev)
        assert lib.cp25_cast_v_bf16t(v.data_ptr(), ctypes.cast(st[2], P), a.B, a.H, a.L, 128, vt.data_ptr(),
                                     stream) == 0

    def run():
        if a.vt:
            nb = 128 ** 0.5 * 1.02
            rc = lib.cp25_attn_fwd_prescaled_vt(q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), a.B, a.H, a.L,
                                                a.L, 128, ctypes.cast(st[0], P), ctypes.cast(st[1], P),
                                                ctypes.cast(st[3], P), nb * c, nb, 1, None, 0, stream)
        elif a.prescaled:
            nb = 128 ** 0.5 * 1.02
            rc = lib.cp25_attn_fwd_prescaled(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), a.B, a.H, a.L, a.L,
                                             128, *[ctypes.cast(s, P) for s in st], nb * c, nb, 1, None, 0, stream)
        elif a.bounded:
            nb = 128 ** 0.5 * 1.02
            rc = lib.cp25_attn_fwd_bounded(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), a.B, a.H, a.L, a.L,
                                           128, *[ctypes.cast(s, P) for s in st], 128 ** -0.5, nb, nb, 1, None, 0,
                                           stream)
        else:
            rc = lib.cp25_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), a.B, a.H, a.L, a.L, 128,
                                   *[ctypes.cast(s, P) for s in st], 128 ** -0.5, stream)
        assert rc == 0, rc

    lib.cp25_attn_probe_set(None, 0)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    lib.cp25_attn_probe_set(ctypes.c_void_p(probe.data_ptr()), a.t0)
    run()
    torch.cuda.synchronize()
    T = probe.cpu().numpy().astype(np.int64).reshape(8, 8, 32, 8)  # wg, wave, tile, stamp
    res = {"L": a.L, "ms": ms, "tflops": 4 * a.B * a.H * a.L * a.L * 128 / ms / 1e9}
    for name, waves in (("A", range(0, 4)), ("B", range(4, 8))):
        t = T[:, list(waves)]
        d = {
            "period": np.diff(t[..., 3], axis=2).mean(),
            "ph1": (t[:, :, 1:, 0] - t[:, :, :-1, 3]).mean(),
            "bar1": (t[..., 1] - t[..., 0]).mean(),
            "ph2": (t[..., 2] - t[..., 1]).mean(),
            "bar2": (t[..., 3] - t[..., 2]).mean(),
        }
        # softmax-phase split: staged LDS write + softmax VALU | load issue for the next staging
        if name == "A":  # stamps 1 -> write_v, softmax -> 5 -> load_tile -> 2
            d["write_softmax"] = (t[:, :, :, 5] - t[:, :, :, 1]).mean()
            d["load_issue"] = (t[:, :, :, 2] - t[:, :, :, 5]).mean()
        else:  # stamps 3 (previous tile) -> write_k, softmax -> 4 -> load_tile -> 0
            d["write_softmax"] = (t[:, :, 1:, 4] - t[:, :, :-1, 3]).mean()
            d["load_issue"] = (t[:, :, 1:, 0] - t[:, :, 1:, 4]).mean()
        # 16x16x32 kernel (stamps 6 / 7 inside the MFMA phase): phase start -> first pair, P.V half, Q K^T half
        if name == "A":
            d["mfma_first_pair"] = (t[:, :, 1:, 6] - t[:, :, :-1, 3]).mean()
        else:
            d["mfma_first_pair"] = (t[..., 6] - t[..., 1]).mean()
        d["mfma_pv_rest"] = (t[..., 7] - t[..., 6]).mean()
        end = t[..., 0] if name == "A" else t[..., 2]
        d["mfma_qk_half"] = (end - t[..., 7]).mean()
        res[name] = {k: round(float(x), 1) for k, x in d.items()}
    res["note"] = ("A: ph1 = MFMA phase, ph2 = softmax; B: ph1 = softmax, ph2 = MFMA (cycles of s_memtime); "
                   "write_softmax / load_issue split the softmax phase")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
