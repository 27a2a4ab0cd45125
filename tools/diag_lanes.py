"""Diagnostic: DiT forward through the per-batch-entry lanes (force_lanes) vs the single B = 2 pass."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))
os.environ.setdefault("CP25_ATTN_SPLIT", "1")

import torch  # noqa: E402

from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict  # noqa: E402
from cosmos_predict2.net_config import tiny_dit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cfg = tiny_dit(num_blocks=2)
    sd = init_state_dict(cfg, seed=3, zero_adaln_out=False)
    net = MinimalV1LVGDiT(cfg, device=dev)
    net.load_state_dict(sd)
    g = torch.Generator().manual_seed(30)
    x = torch.randn(2, 16, 3, 16, 32, generator=g).to(dev)
    t = torch.tensor([[0.1, 877.0, 877.0], [0.1, 877.0, 877.0]], device=dev)
    ctx = torch.randn(2, 512, cfg.crossattn_proj_in_channels, generator=g).to(dev, torch.bfloat16)
    a = net(x, t, ctx)
    net.force_lanes = True
    b = net(x, t, ctx)
    torch.cuda.synchronize()
    for i in range(2):
        e = ((a[i] - b[i]).norm() / a[i].norm()).item()
        print(f"batch {i}: lanes vs single pass rel-L2 {e:.3e}, equal={torch.equal(a[i], b[i])}")


if __name__ == "__main__":
    main()
