"""Diagnostic: fused CFG-batched DiT (B=2, shared input rows) vs two single-branch forwards."""
import sys, dataclasses
sys.path[:0] = [".", "cosmos-predict2.5_amd"]
import torch
from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict, Geometry
from cosmos_predict2.net_config import tiny_dit
from cosmos_predict2 import _native as N
from cosmos_predict2.model import to_patch_layout

dev = torch.device("cuda:0")
cfg = tiny_dit(num_blocks=2)
sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=1, zero_adaln_out=False).items()}
net = MinimalV1LVGDiT(cfg, device=dev); net.load_state_dict(sd)
T, H, W = 3, 16, 16
g = torch.Generator().manual_seed(20)
x = torch.randn(1, 16, T, H, W, generator=g)
c1 = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
c2 = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
mask = torch.zeros(1, 1, T, H, W); mask[:, :, :1] = 1
t = torch.tensor([[0.1, 877.0, 877.0]])
outs = []
for c in (c1, c2):
    outs.append(net(x.to(dev).to(torch.bfloat16), t.to(dev), c.to(dev), condition_video_input_mask_B_C_T_H_W=mask.to(dev)))
# fused
geo = Geometry(T=T, Hp=H // 2, Wp=W // 2, tok0=0, n_tok=T * H * W // 4)
xs = to_patch_layout(x[0].to(dev))
fm = torch.tensor([1.0, 0, 0], device=dev)
rows = N.patchify(xs, None, fm, None, tok0=0, hw=geo.hw)
ctx = net.prepare_context(torch.cat([c1, c2]).to(dev))
tb = (t.to(dev) * cfg.timestep_scale).expand(2, T).contiguous()
o2 = net.forward_tokens(rows.view(geo.n_tok, 1, -1), tb, ctx, geo)  # [L, 2, 64]
for b in range(2):
    ob = to_patch_layout(outs[b][0])
    print("branch", b, "rel diff fused vs single:", ((o2[:, b] - ob).norm() / ob.norm()).item())
print("cond vs uncond rel diff:", ((outs[0] - outs[1]).norm() / outs[0].norm()).item())
