"""Debug aid for gemm_nt_4w: error map of cp25_gemm_select(1) against the fp32 product on small shapes."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))
import torch
from cosmos_predict2 import _native as N
dev = torch.device("cuda:0")
for (M, Nn, K) in ((256, 256, 128), (256, 256, 256), (512, 256, 128)):
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(Nn, K, generator=g, device=dev) * K ** -0.5).to(torch.bfloat16)
    ref = (a.float() @ w.float().t())
    N.gemm_select(0); o8 = N.gemm_epi(a, w).float()
    N.gemm_select(1); o4 = N.gemm_epi(a, w).float()
    torch.cuda.synchronize()
    e8 = (o8 - ref).abs(); e4 = (o4 - ref).abs()
    print(M, Nn, K, "8ph max err", e8.max().item(), "4w max err", e4.max().item())
    bad = (e4 > 0.05)
    blk = bad.view(M // 16, 16, Nn // 16, 16).any(3).any(1).int()
    print("bad 16x16 blocks (rows of row-blocks):")
    for r in range(blk.shape[0]):
        print("".join("X" if x else "." for x in blk[r].tolist()))
    # is the 4w output some other product? try candidates
    rows_bad = bad.any(1).nonzero().flatten().tolist()[:8]
    print("first bad rows", rows_bad, "cols", bad.any(0).nonzero().flatten().tolist()[:8])
    if rows_bad:
        r = rows_bad[0]; c = bad[r].nonzero().flatten()[0].item()
        print("r,c", r, c, "ref", ref[r, c].item(), "4w", o4[r, c].item())
        # candidate: partial K sums
        for k0, k1 in ((0, 32), (32, 64), (0, 64), (64, 128), (0, K - 32)):
            if k1 <= K:
                print("  K", k0, k1, (a[r, k0:k1].float() @ w[c, k0:k1].float()).item())
