"""Lab diagnostics for attn_fwd_w64 vs attn_fwd_m16 (round 6): error vs fp32 of both forms and where they differ."""
import json
import sys

import torch

sys.path.insert(0, "cosmos-predict2.5_amd")
from cosmos_predict2 import _native as N  # noqa: E402

LOG2E = 1.4426950408889634
C = 128 ** -0.5 * LOG2E
dev = torch.device("cuda:0")


def ref(q, k, v):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    p = torch.softmax(torch.matmul(qf, kf.transpose(-1, -2)) / LOG2E, dim=-1)
    return torch.matmul(p, vf).transpose(1, 2)


def case(B, H, Lq, Lk, n_split, mode, kind="randn"):
    g = torch.Generator(device="cpu").manual_seed(1)
    q = torch.randn(B, Lq, H, 128, generator=g)
    q = (q * torch.rsqrt(q.pow(2).mean(-1, keepdim=True)) * C).to(torch.bfloat16).to(dev)
    k = torch.randn(B, Lk, H, 128, generator=g)
    k = (k * torch.rsqrt(k.pow(2).mean(-1, keepdim=True))).to(torch.bfloat16).to(dev)
    v = torch.randn(B, Lk, H, 128, generator=g).to(dev, torch.bfloat16)
    if kind == "vones":
        v = torch.ones_like(v)
    if kind == "vcol":  # v[key, d] = d: any key gives the column index
        v = torch.arange(128, device=dev).float().expand(B, Lk, H, 128).to(torch.bfloat16).contiguous()
    if kind == "vkey":  # v[key, d] = key (small Lk): P-weighted key index
        v = (torch.arange(Lk, device=dev).float() / Lk)[None, :, None, None].expand(B, Lk, H, 128).to(torch.bfloat16).contiguous()
    nb = (q.float().norm(dim=-1).max().item() * 1.01, k.float().norm(dim=-1).max().item() * 1.01) if mode == "zero" else None
    r = ref(q, k, v)
    out = {}
    for form in (0, 1):
        N.attn_self_select(form)
        o = N.attn_fwd(q, k, v, prescaled=True, n_split=n_split, norm_bounds=nb)
        torch.cuda.synchronize()
        out[form] = o.float()
    N.attn_self_select(1)
    a, b = out[0], out[1]
    d = (a - b).abs()
    res = {"shape": [B, H, Lq, Lk, n_split, mode, kind],
           "m16_vs_fp32": ((a - r).norm() / r.norm()).item(), "w64_vs_fp32": ((b - r).norm() / r.norm()).item(),
           "equal": bool(torch.equal(a, b)), "maxdiff": d.max().item(),
           "nan_w64": int(torch.isnan(b).sum().item())}
    rows = d.amax(dim=(0, 2, 3))  # per query row
    bad = torch.nonzero(rows > 0).flatten().tolist()
    res["bad_rows_n"] = len(bad)
    res["bad_rows_head"] = bad[:16]
    if bad:
        res["bad_rows_mod64"] = sorted(set(x % 64 for x in bad))[:40]
        res["bad_rows_mod256_div64"] = sorted(set((x % 256) // 64 for x in bad))
        cols = d.amax(dim=(0, 1, 2))
        res["bad_cols"] = torch.nonzero(cols > 0).flatten().tolist()[:40]
        x = bad[0]
        res["row0_w64"] = b[0, x, 0, :8].tolist()
        res["row0_m16"] = a[0, x, 0, :8].tolist()
        res["row0_ref"] = r[0, x, 0, :8].tolist()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        N._LIB_PATH = sys.argv[1]
    case(1, 1, 256, 4160, 1, "zero", "vcol")
    case(1, 1, 256, 4160, 1, "zero", "vones")
    case(1, 1, 256, 4160, 1, "zero", "vkey")
    case(1, 1, 256, 4160, 1, "zero")
    case(1, 1, 256, 4224, 1, "zero")
    case(1, 1, 256, 4100, 1, "zero")
    case(1, 1, 256, 4160, 1, "online")
    case(1, 2, 513, 4100, 1, "zero")
