"""CPU estimate of what fp8 attention operands cost at full depth, before building them: the 28-block 2B
forward at config-1 geometry (oracle/dit.py, bf16 reference arithmetic) with its SDPA replaced by emulations,
each compared with the fp32 truth (the same test geometry and seeds as tests/test_parity_depth_gpu.py).

  qk   : Q K^T on e4m3 copies of q*c*4 and k/4 (what cp25_attn_fwd_prescaled_fp8qk computes)
  qkpv : + P = exp2(S - (b_row - 15)) as e5m2 (b_row = the row's Cauchy-Schwarz score bound, so P <= 2^15 fits
         e5m2 without overflow whatever the data) and V as e4m3 with a per-tensor scale
  pvc  : as qkpv with one constant shift per launch, b = max|q c| max|k| - 15 (what the kernel builds: the shift
         enters as the Q K^T MFMA chain's initial C)
  pv43 : + P as e4m3 with the shift b_row - 8 (P <= 256 < 448) instead: underflows whole rows (NaN)
  pvs  : as pvc, but the e5m2 byte of P made in one integer convert, n = round(4 (S - shift) + 60) clamped to
         [0, 123] and read as e5m2 (2^(n/4 - 15) with a linear mantissa: exp2 never evaluated), the row sums
         taken over those P (an all-ones V^T row in the P.V MFMA)

usage: python tools/sim_fp8_attention_depth.py  (about 10 CPU-minutes)
"""
import dataclasses
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

from cosmos_predict2.dit import init_state_dict  # noqa: E402
from cosmos_predict2.net_config import DIT_2B  # noqa: E402
from oracle import dit as odit  # noqa: E402

C = 128 ** -0.5 * 1.4426950408889634
E4, E5 = torch.float8_e4m3fn, torch.float8_e5m2


def make_sdpa(mode):
    def sdpa(q, k, v, chunk=4096):
        B, Lq, H, D = q.shape
        qs = (q.float() * C).to(torch.bfloat16).float()
        q8 = (qs * 4).clamp(-448, 448).to(E4).float() / 4
        k8 = (k.float() / 4).clamp(-448, 448).to(E4).float() * 4
        qf, kf, vf = (t.transpose(1, 2) for t in (q8, k8, v.float()))
        s = qf @ kf.transpose(-1, -2)  # log2 units
        if mode == "qk":
            p = torch.exp2(s - s.amax(-1, keepdim=True))
            o = (p.to(torch.bfloat16).float() @ vf) / p.sum(-1, keepdim=True)
        else:
            b = qs.transpose(1, 2).norm(dim=-1, keepdim=True) * k.float().norm(dim=-1).amax() * 1.0
            if mode in ("pvc", "pvs"):
                b = b.amax()
            top, fmt = (15.0, E5) if mode in ("qkpv", "pvc", "pvs") else (8.0, E4)
            if mode == "pvs":
                n = torch.round(4 * (s - (b - top)) + 60).clamp(0, 123).to(torch.uint8)
                p = n.view(E5).float()
            else:
                p = torch.exp2(s - (b - top)).to(fmt).float()
            vsc = vf.abs().amax().clamp(min=1e-30) / 448.0
            v8 = (vf / vsc).to(E4).float() * vsc
            o = (p @ v8) / p.sum(-1, keepdim=True)
        return o.transpose(1, 2).reshape(B, Lq, H * D).to(odit.act_dtype())
    return sdpa


def main():
    cfg = DIT_2B
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=11, zero_adaln_out=False).items()}
    g = torch.Generator().manual_seed(31)
    T, H, W = 3, 32, 32
    x = torch.randn(1, 16, T, H, W, generator=g)
    mask = torch.zeros(1, 1, T, H, W)
    mask[:, :, :1] = 1
    t = torch.tensor([[0.1, 877.0, 877.0]])
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    c = dataclasses.asdict(cfg)
    with odit.fp32_truth():
        truth = odit.dit_forward(c, sd, x, t, ctx, mask)
    rel = lambda a: ((a.float() - truth).norm() / truth.norm()).item()  # noqa: E731
    ref = odit.dit_forward(c, sd, x, t, ctx, mask)
    print(f"bf16 reference arithmetic vs fp32 truth: {rel(ref):.3e}", flush=True)
    orig = odit.sdpa
    for mode in sys.argv[1:] or ("qk", "qkpv", "pvc", "pv43"):
        odit.sdpa = make_sdpa(mode)
        try:
            out = odit.dit_forward(c, sd, x, t, ctx, mask)
        finally:
            odit.sdpa = orig
        print(f"{mode}: vs fp32 truth {rel(out):.3e}", flush=True)


if __name__ == "__main__":
    main()
