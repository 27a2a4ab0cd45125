"""Lab A/B (round 6): does the magnitude of P move the self-attention's power-limited clock? With trained-size q/k
norm weights (uniform in [0.5, 3]) the DiT's self-attention runs the online-max loop (P <= 2^24, the row max near 1),
and the zero-shift loop on the same data (P = 2^S up to ~2^30) measured no faster than it. At the metric
launch (B 2, H 16, L 109 120, the DiT's fused in-kernel q-norm form) this times, alternating in one process:
  zero    the product's zero-shift loop on the trained-weight data (bounds passed small enough to select it; the
          data's true score bound is ~64 in log2 units, inside the loop's 96)
  online  the product's online-max loop (the weight bounds, as the DiT passes them)
  dshift  tools/lab/libcp25_dshift.so's fixed-shift loop with the shift the row's whole data-tight bound,
          floor(|q_row| max|k|): P <= 2, an integer shift, so its output is bit-identical to `zero`
  unit    the product's zero-shift loop on unit-weight data (the headline's case)
One JSON line: ms lists and medians per form, and the bit-identity of dshift vs zero.
  python tools/lab/ab_shift_power.py [--rounds 4] [--iters 4]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402


def data(dev, L, B, H, lo, hi, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    D = H * 128
    buf = torch.randn(L, B, 3 * D, device=dev, generator=g).to(torch.bfloat16)
    q, k, v = (buf[:, :, i * D:(i + 1) * D].view(L, B, H, 128).transpose(0, 1) for i in range(3))
    w = lo + (hi - lo) * torch.rand(128, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
    k.copy_((k.float() * torch.rsqrt(k.float().pow(2).mean(-1, keepdim=True) + 1e-6) * w).to(torch.bfloat16))
    c = 128 ** -0.5 * 1.4426950408889634
    ang = torch.rand(L, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(6)) * 50.0
    qn = dict(weight=w.to(torch.bfloat16), cos=torch.cos(ang).contiguous(), sin=torch.sin(ang).contiguous(), out_scale=c)
    wb = 128 ** 0.5 * float(w.abs().max()) * 1.02
    kd = float(k.float().norm(dim=-1).max()) * 1.001  # data-tight key bound
    return buf, q, k, v, qn, (wb * c, wb), kd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    L, B, H = 109120, 2, 16
    prod = N.load_library()
    N._lib, N._LIB_PATH = None, os.path.join(ROOT, "tools", "lab", "libcp25_dshift.so")
    lab = N.load_library()
    N._lib = prod
    _, q, k, v, qn, wbounds, kd = data(dev, L, B, H, 0.5, 3.0, 0)
    _, qu, ku, vu, qnu, ubounds, _ = data(dev, L, B, H, 1.0, 1.0, 1)
    o = torch.empty(B, L, H, 128, device=dev, dtype=torch.bfloat16)
    forms = {
        "zero": (prod, (q, k, v, qn), (1e-3, kd)),          # product 1e-3 * kd <= 96: zero-shift mode
        "online": (prod, (q, k, v, qn), wbounds),           # weight bounds ~147 > 98: online max
        "dshift": (lab, (q, k, v, qn), (97.0 / kd, kd)),    # product 97: fixed-shift mode, the lab's whole-bound shift
        "unit": (prod, (qu, ku, vu, qnu), ubounds),         # unit weights: zero shift
        # unit weights, the lab's whole-bound shift from the weight-based key bound (fixed-shift mode selected by a
        # q bound of 97 / kb): floor(|q_row| kb) <= 17 here, P <= 2
        "unit_dshift": (lab, (qu, ku, vu, qnu), (97.0 / ubounds[1], ubounds[1])),
    }
    names = {}
    outs = {}

    def run(f):
        lib, (qq, kk, vv, qn_), nb = forms[f]
        N._lib = lib
        N.attn_fwd(qq, kk, vv, out=o, norm_bounds=nb, prescaled=True, q_norm=qn_)
        return nb

    for f in forms:
        nb = run(f)
        torch.cuda.synchronize()
        outs[f] = o.clone()
        names[f] = N.attn_kernel_name(L, norm_bounds=nb, prescaled=True)
    same = bool(torch.equal(outs["zero"], outs["dshift"]))

    def rel(x, y):
        return float((outs[x].float() - outs[y].float()).norm() / outs[y].float().norm())
    rels = {"online_vs_zero": rel("online", "zero"), "dshift_vs_zero": rel("dshift", "zero"),
            "unit_dshift_vs_unit": rel("unit_dshift", "unit"), "unit_dshift_equal_unit": bool(torch.equal(
                outs["unit_dshift"], outs["unit"]))}
    del outs
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = {f: [] for f in forms}
    fl = list(forms)
    for r in range(a.rounds):
        for f in fl[r % len(fl):] + fl[:r % len(fl)]:
            run(f)
            e0.record(st)
            for _ in range(a.iters):
                run(f)
            e1.record(st)
            torch.cuda.synchronize()
            ms[f].append(round(e0.elapsed_time(e1) / a.iters, 3))
    N._lib = prod
    med = {f: sorted(x)[len(x) // 2] for f, x in ms.items()}
    print(json.dumps({"ms": ms, "median": med, "kernels": names, "dshift_bit_identical_to_zero": same,
                      "rel_l2": rels, "data_tight_k_bound": kd, "weight_bounds": wbounds}))


if __name__ == "__main__":
    main()
