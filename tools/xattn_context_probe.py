"""Why the text cross-attention runs slower inside the DiT than alone: the same launch (the DiT's layout, B = 2,
109 120 queries, 512 text keys, prescaled zero-shift form) timed with HIP events (a) back to back, (b) each right after
one full self-attention launch, (c) each right after an MLP1 GEMM, (d) with the query read at batch stride 0 (block
0's CFG-shared query), (e) right after the q RMSNorm / the cross-q GEMM + norm that precede it in the DiT. One JSON line.
usage: python tools/xattn_context_probe.py [--reps 10]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402


def rms_rows(t):
    return (t.float() * torch.rsqrt(t.float().pow(2).mean(-1, keepdim=True) + 1e-6)).to(torch.bfloat16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    L, B, H, hd, Lc = 109120, 2, 16, 128, 512
    D = H * hd
    c = hd ** -0.5 * 1.4426950408889634
    bnd = (hd ** 0.5 * c * 1.001, hd ** 0.5 * 1.001)
    # cross-attention operands as the DiT holds them: q rows of a [n, B, D] buffer, text K/V [B, 512, H, hd]
    qc = (rms_rows(torch.randn(L, B, H, hd, device=dev, generator=g)).float() * c).to(torch.bfloat16)
    kc = rms_rows(torch.randn(B, Lc, H, hd, device=dev, generator=g))
    vc = torch.randn(B, Lc, H, hd, device=dev, generator=g).to(torch.bfloat16)
    oc = torch.empty(L, B, H, hd, device=dev, dtype=torch.bfloat16)
    q1 = qc[:, :1].expand(L, B, H, hd)  # block 0: one query shared by the CFG pair (batch stride 0)

    def xattn(q=qc):
        N.attn_fwd(q.transpose(0, 1), kc, vc, out=oc.transpose(0, 1), norm_bounds=bnd, prescaled=True)

    # a full self-attention launch (fused QKV layout, prescaled bounded form)
    buf = torch.randn(L, B, 3 * D, device=dev, generator=g).to(torch.bfloat16)
    qs, ks, vs = (buf[:, :, i * D:(i + 1) * D].view(L, B, H, hd) for i in range(3))
    qs.copy_((rms_rows(qs).float() * c).to(torch.bfloat16))
    ks.copy_(rms_rows(ks))
    os_ = torch.empty(L, B, H, hd, device=dev, dtype=torch.bfloat16)

    def self_attn():
        N.attn_fwd(qs.transpose(0, 1), ks.transpose(0, 1), vs.transpose(0, 1), out=os_.transpose(0, 1),
                   norm_bounds=bnd, prescaled=True)

    x = torch.randn(L * B, D, device=dev, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(4 * D, D, device=dev, generator=g) * D ** -0.5).to(torch.bfloat16)

    def mlp1():
        N.gemm_epi(x, w1, epilogue=N.EPI_GELU)

    wq = torch.ones(hd, device=dev, dtype=torch.bfloat16)
    qflat = qc.view(L * B, D)

    def qnorm():  # the q RMSNorm (+ the prescale) that precedes the launch in the DiT (in place, idempotent here)
        N.head_rmsnorm_rope(qflat, n_rows=L * B, B=B, H=H, head_off=0, weight=wq, out_scale=c)

    def xq_then_qnorm():  # the cross-q GEMM writing q, then its norm (the DiT's exact sequence)
        N.gemm_epi(x, w1[:D], out=qflat)
        qnorm()

    def timed_after(pre, q=qc):
        ts = []
        for _ in range(a.reps):
            if pre is not None:
                pre()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            xattn(q)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return ts

    xattn()
    self_attn()
    mlp1()
    torch.cuda.synchronize()
    rec = {}
    for name, pre, q in (("alone", None, qc), ("after_self_attention", self_attn, qc), ("after_mlp1", mlp1, qc),
                         ("alone_shared_q", None, q1), ("after_self_attention_shared_q", self_attn, q1),
                         ("after_qnorm", qnorm, qc), ("after_crossq_gemm_and_qnorm", xq_then_qnorm, qc),
                         ("alone_again", None, qc)):
        ts = timed_after(pre, q)
        rec[name] = {"mean_ms": sum(ts) / len(ts), "min_ms": min(ts), "max_ms": max(ts)}
    # back to back without host syncs between launches
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        xattn()
    e1.record()
    torch.cuda.synchronize()
    rec["back_to_back_mean_ms"] = e0.elapsed_time(e1) / a.reps
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
