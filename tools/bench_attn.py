"""Micro-benchmark of cp25_attn_fwd at the DiT's shapes (timed with HIP events on the launch stream).

usage: python tools/bench_attn.py [--L 109120] [--B 2] [--H 16] [--iters 5] [--bounded]
Prints one JSON line per shape: ms per launch and TFLOP/s (4*B*H*Lq*Lk*D algorithmic FLOP).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402


def probe_report(T, clk=None):
    """Phase anatomy of the attn_fwd_m16 loop from the lab probe's stamps T[wg][wave][tile][k] (s_memtime cycles).
    Waves w and w + 4 share a SIMD. Per tile t: phase X = group A's MFMA phase (A0 -> A1: P.V(t), Q K^T(t+1)) beside
    group B's softmax(t) (B0 -> B1), released at A2; phase Y = B's MFMA phase (B2 -> B3) beside A's softmax(t+1)
    (A2 -> A3), released at the next A0. 68 MFMAs of 16 cycles = 1088 cycles of pipe per MFMA phase."""
    import numpy as np
    T = T.astype(np.int64)
    A, Bw = T[:, 0:4], T[:, 4:8]
    A0, A1, A2, A3 = (A[..., i] for i in range(4))
    B0, B1, B2, B3 = (Bw[..., i] for i in range(4))
    nxt = A0[:, :, 1:]
    sl = (slice(None), slice(None), slice(0, -1))
    r = {}

    def m(x):
        return round(float(np.median(x)), 1)
    r["period"] = m(nxt - A0[sl])
    r["X_len"] = m(A2[sl] - A0[sl])
    r["Y_len"] = m(nxt - A2[sl])
    r["A_mfma_span"] = m(A1 - A0)
    r["B_mfma_span"] = m(B3 - B2)
    r["B_softmax_span"] = m(B1 - B0)
    r["A_softmax_span"] = m(A3 - A2)
    r["X_overrun_softmax_after_mfma"] = m(B1 - A1)
    r["Y_overrun_softmax_after_mfma"] = m(A3[sl] - B3[sl])
    r["X_release_after_last"] = m(A2 - np.maximum(A1, B1))
    r["Y_release_after_last"] = m(nxt - np.maximum(A3[sl], B3[sl]))
    r["X_open_skew_B0_minus_A0"] = m(B0 - A0)
    r["Y_open_skew_B2_minus_A2"] = m(B2 - A2)
    idle = (nxt - A0[sl]) - (A1 - A0)[sl] - (B3 - B2)[sl]
    r["mfma_idle_per_tile"] = m(idle)
    # barrier anatomy over the whole workgroup: arrivals = the MFMA waves' last MFMA (A1 / B3) and the softmax waves'
    # finished work (B1 / A3); release = the earliest opening stamp after the barrier (A2 / next A0)
    arr_X = np.concatenate([A1, B1], axis=1)          # [wg, 8, tile]
    arr_Y = np.concatenate([A3, B3], axis=1)[sl]
    rel_X = np.minimum(A2.min(1), B2.min(1))          # [wg, tile]
    rel_Y = np.minimum(A0.min(1), B0.min(1))[:, 1:]
    r["X_release_after_last_of_8"] = m(rel_X - arr_X.max(1))
    r["Y_release_after_last_of_8"] = m(rel_Y - arr_Y.max(1))
    r["X_mfma_end_skew_over_simds"] = m(A1.max(1) - A1.min(1))  # group A's 4 MFMA waves
    r["Y_mfma_end_skew_over_simds"] = m(B3.max(1) - B3.min(1))
    r["X_last_arrival_is_mfma_wave"] = round(float((A1.max(1) >= B1.max(1)).mean()), 3)
    r["Y_last_arrival_is_mfma_wave"] = round(float((B3[sl].max(1) >= A3[sl].max(1)).mean()), 3)
    r["mfma_busy_share"] = round(float(np.median(((A1 - A0)[sl] + (B3 - B2)[sl]) / (nxt - A0[sl]))), 4)
    if clk is not None:  # loop start / end: s_memtime (shader cycles) and s_memrealtime (100 MHz) per wave
        clk = clk.astype(np.int64)
        r["clock_ghz"] = round(float(np.median((clk[..., 2] - clk[..., 0]) / (clk[..., 3] - clk[..., 1]))) * 0.1, 4)
        r["loop_cycles"] = m(clk[..., 2] - clk[..., 0])
        if clk.shape[-1] > 4:
            r["rescale_tiles_per_wave"] = round(float(clk[..., 4].mean()), 2)
    r["note"] = "medians over workgroups x SIMDs x tiles, s_memtime cycles, each wait-form stamp ~40 cycles"
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=109120)
    ap.add_argument("--Lk", type=int, default=0)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--fused", action="store_true",
                    help="q/k/v as strided views of a token-major [L, B, 3*H*128] QKV buffer (the DiT's layout)")
    ap.add_argument("--zeros", action="store_true", help="zero-filled inputs (DVFS reference point)")
    ap.add_argument("--split", type=int, default=0, help="key-range split (0 = the library's plan)")
    ap.add_argument("--bounded", action="store_true",
                    help="RMS-normalised q/k rows (as the DiT's q/k norm leaves them) and their norm bounds: the "
                         "bounded-shift softmax (cp25_attn_fwd_bounded)")
    ap.add_argument("--normed", action="store_true", help="RMS-normalised q/k rows without passing the bounds")
    ap.add_argument("--wrange", default="1,1", help="lo,hi: q/k RMSNorm weights uniform in [lo, hi] (seeded; 1,1 = the "
                    "unit init weights); --bounded passes the DiT's weight bounds sqrt(128) max|w| 1.02")
    ap.add_argument("--prescaled", action="store_true",
                    help="with --bounded: q carries scale*log2(e) (the DiT's default form, cp25_attn_fwd_prescaled)")
    ap.add_argument("--fp8qk", action="store_true",
                    help="with --prescaled: Q K^T on e4m3 copies of q*4 and k/4 (cp25_attn_fwd_prescaled_fp8qk)")
    ap.add_argument("--fp8pv", action="store_true",
                    help="with --fp8qk: P.V on e5m2 P and e4m3 V too (cp25_attn_fwd_prescaled_fp8)")
    ap.add_argument("--qnorm", action="store_true",
                    help="with --bounded --prescaled: q stays the raw projection and the kernel applies the q RMSNorm "
                         "+ RoPE + prescale itself (cp25_attn_fwd_prescaled_qnorm, the DiT's default since round 4)")
    ap.add_argument("--lib", default="", help="lab build of libcp25.so to load instead of the in-tree one")
    ap.add_argument("--self-form", type=int, default=-1,
                    help="w64 lab library (tools/lab/w64/build_lab.sh, with --lib): prescaled self-attention form, 0 attn_fwd_m16, 1 w64 in the zero / fixed modes, 2 w64 in all (cp25_attn_self_select)")
    ap.add_argument("--ab", type=int, default=0,
                    help="A/B: after the timing, N more rounds alternating attn_fwd_m16 / attn_fwd_w64 launches "
                         "(iters each), reported as ms lists per form")
    ap.add_argument("--ab-libs", default="",
                    help="comma-separated lab builds of libcp25.so: after the timing, --ab rounds alternating the "
                         "loaded library and these (rotating order, iters launches each), reported as ms lists per "
                         "library, with each library's output compared bit for bit with the first's")
    ap.add_argument("--probe", type=int, default=-1,
                    help="with a -DCP25_ATTN_PROBE lab build: after the timing, one more launch records s_memtime "
                         "stamps of tiles probe .. probe + 31 in the first --probe-wg workgroups (probe_report)")
    ap.add_argument("--probe-wg", type=int, default=64)
    ap.add_argument("--probe-dump", default="", help="save the raw probe stamps (.npy) here")
    ap.add_argument("--force-online", action="store_true",
                    help="with --bounded: pass a 10x larger q bound, so the online-max form runs on data the zero-shift "
                         "form would take (the online form's cost on the same data)")
    a = ap.parse_args()
    if a.lib:
        N._LIB_PATH = a.lib
    if a.self_form >= 0:
        N.attn_self_select(a.self_form)
    dev = torch.device("cuda:0")
    Lk = a.Lk or a.L
    g = torch.Generator(device=dev).manual_seed(0)
    if a.fused:
        assert Lk == a.L
        D = a.H * 128
        buf = torch.randn(a.L, a.B, 3 * D, device=dev, generator=g).to(torch.bfloat16)
        q, k, v = (buf[:, :, i * D:(i + 1) * D].view(a.L, a.B, a.H, 128).transpose(0, 1) for i in range(3))
    else:
        q = torch.randn(a.B, a.L, a.H, 128, device=dev, generator=g).to(torch.bfloat16)
        k = torch.randn(a.B, Lk, a.H, 128, device=dev, generator=g).to(torch.bfloat16)
        v = torch.randn(a.B, Lk, a.H, 128, device=dev, generator=g).to(torch.bfloat16)
    if a.zeros:
        for t in (q, k, v):
            t.zero_()
    nb = None
    q_raw = q.clone() if a.qnorm else None
    if a.bounded or a.normed:
        lo, hi = (float(x) for x in a.wrange.split(","))
        w = lo + (hi - lo) * torch.rand(128, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
        for t in (q, k):  # RMSNorm with weight w, in place, per head row
            t.copy_((t.float() * torch.rsqrt(t.float().pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16))
        wb = 128 ** 0.5 * float(w.abs().max()) * 1.02
        nb = (wb, wb) if a.bounded else None
    pre = {}
    if a.prescaled:
        c = 128 ** -0.5 * 1.4426950408889634
        q.copy_((q.float() * c).to(torch.bfloat16))
        nb = (nb[0] * c, nb[1]) if nb else None
        pre = dict(prescaled=True)
        if a.qnorm:
            assert a.bounded and not a.fp8qk, "--qnorm goes with --bounded --prescaled (bf16)"
            ang = torch.rand(a.L, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(6)) * 50.0
            q.copy_(q_raw)
            pre["q_norm"] = dict(weight=w.to(torch.bfloat16), cos=torch.cos(ang).contiguous(),
                                 sin=torch.sin(ang).contiguous(), out_scale=c)
        if a.fp8qk:
            if a.fused:
                cols = [buf.view(a.L * a.B, 3 * D)[:, i * D:(i + 1) * D] for i in range(2)]
                q8, k8 = (N.cast_fp8(cols[i], s).view(a.L, a.B, a.H, 128).transpose(0, 1)
                          for i, s in ((0, 4.0), (1, 0.25)))
            else:
                q8 = N.cast_fp8(q.reshape(-1, 128), 4.0).view(q.shape)
                k8 = N.cast_fp8(k.reshape(-1, 128), 0.25).view(k.shape)
            pre["fp8_qk"] = (q8, k8)
            if a.fp8pv:
                pre["fp8_v"] = N.cast_v_fp8t(v)
    if a.force_online:
        assert nb, "--force-online goes with --bounded"
        nb = (nb[0] * 10.0, nb[1])
    # correctness of the loaded build on a small shape (ragged length) vs fp32 math
    gc = torch.Generator(device=dev).manual_seed(1)
    qc, kc, vc = (torch.randn(1, 1000, 2, 128, device=dev, generator=gc).to(torch.bfloat16) for _ in range(3))
    ref = torch.softmax(torch.einsum("bqhd,bkhd->bhqk", qc.float(), kc.float()) * 128 ** -0.5, -1)
    ref = torch.einsum("bhqk,bkhd->bqhd", ref, vc.float())
    ncb = (qc.float().norm(dim=-1).max().item(), kc.float().norm(dim=-1).max().item()) if a.bounded else None
    oc = N.attn_fwd(qc, kc, vc, n_split=1, norm_bounds=ncb).float()
    check = float((oc - ref).norm() / ref.norm())
    ns = a.split or None  # None: the library's plan, with its tail split where it pays
    o = N.attn_fwd(q, k, v, n_split=ns, norm_bounds=nb, **pre)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.iters):
        N.attn_fwd(q, k, v, out=o, n_split=ns, norm_bounds=nb, **pre)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flop = 4.0 * a.B * a.H * a.L * Lk * 128
    ab = None
    if a.ab > 0 and not a.ab_libs:
        ab = {"m16": [], "w64": []}
        prev = N.attn_self_select(0)
        for _ in range(a.ab):
            for form, key in ((0, "m16"), (1, "w64")):
                N.attn_self_select(form)
                N.attn_fwd(q, k, v, out=o, n_split=ns, norm_bounds=nb, **pre)
                e0.record(st)
                for _ in range(a.iters):
                    N.attn_fwd(q, k, v, out=o, n_split=ns, norm_bounds=nb, **pre)
                e1.record(st)
                torch.cuda.synchronize()
                ab[key].append(round(e0.elapsed_time(e1) / a.iters, 3))
        N.attn_self_select(prev)
    if a.ab_libs:
        libs = {os.path.basename(a.lib) or "libcp25.so": N.load_library()}
        for path in a.ab_libs.split(","):
            N._lib, N._LIB_PATH = None, path
            libs[os.path.basename(path)] = N.load_library()
        names = list(libs)
        ab, same, o0 = {n: [] for n in names}, {}, None
        for r in range(max(a.ab, 1)):
            for n in names[r % len(names):] + names[:r % len(names)]:
                N._lib = libs[n]
                N.attn_fwd(q, k, v, out=o, n_split=ns, norm_bounds=nb, **pre)
                torch.cuda.synchronize()
                if r == 0:
                    if o0 is None:
                        o0 = o.clone()
                    same[n] = bool(torch.equal(o, o0))
                e0.record(st)
                for _ in range(a.iters):
                    N.attn_fwd(q, k, v, out=o, n_split=ns, norm_bounds=nb, **pre)
                e1.record(st)
                torch.cuda.synchronize()
                ab[n].append(round(e0.elapsed_time(e1) / a.iters, 3))
        N._lib = libs[names[0]]
        ab = {"ms": ab, "median": {n: sorted(v_)[len(v_) // 2] for n, v_ in ab.items()}, "bit_identical": same}
    probe = None
    if a.probe >= 0:
        import ctypes
        lib = N.load_library()
        lib.cp25_attn_probe_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        buf_p = torch.zeros(a.probe_wg * 8 * (32 * 4 + 8), dtype=torch.int64, device=dev)
        lib.cp25_attn_probe_set(ctypes.c_void_p(buf_p.data_ptr()), a.probe, a.probe_wg)
        N.attn_fwd(q, k, v, out=o, n_split=ns, norm_bounds=nb, **pre)
        torch.cuda.synchronize()
        lib.cp25_attn_probe_set(None, 0, 0)
        pb = buf_p.cpu().numpy()
        if a.probe_dump:
            import numpy as np
            np.save(a.probe_dump, pb)
        n_t = a.probe_wg * 8 * 128
        probe = probe_report(pb[:n_t].reshape(a.probe_wg, 8, 32, 4), pb[n_t:].reshape(a.probe_wg, 8, 8))
    print(json.dumps({"kernel": "attn_fwd", "B": a.B, "H": a.H, "Lq": a.L, "Lk": Lk, "fused": a.fused,
                      "zeros": a.zeros, "bounded": a.bounded, "prescaled": a.prescaled, "fp8qk": a.fp8qk, "fp8pv": a.fp8pv, "qnorm": a.qnorm, "force_online": a.force_online, "normed": a.normed or a.bounded, "wrange": a.wrange, "split": ns or N.attn_plan(a.B, a.H, a.L, Lk), "iters": a.iters, "lib": os.path.basename(a.lib) or "libcp25.so", "ms": ms,
                      "tflops": flop / ms / 1e9, "check_rel_l2": check, "kernel_name": N.attn_kernel_name(Lk, norm_bounds=nb, prescaled=a.prescaled), **({"probe": probe} if probe else {}), **({"ab_ms": ab} if ab else {})}))


if __name__ == "__main__":
    main()
