"""The cross-view multi-view net (MultiViewCrossDiT, predict2_multiview/networks/multiview_cross_dit.py:502-869) on the
device against the oracle's restatement (oracle/dit.py): per-view self-attention, the cross-view sub-layer (affine
LayerNorm on cp25_layer_norm, one q|k|v GEMM, neighbour K/V gathered per frame, un-gated residual through the gated-
residual GEMM with a unit gate), the per-view AdaLN terms (cp25_gemm_f32). Tolerance rel-L2 <= 1e-2 of the fp32
output, as the other DiT forwards (tests/test_dit_gpu.py): bf16 rounding order and the attention's bf16 P.
Also cp25_layer_norm against torch's affine LayerNorm on the same bf16 rows."""
import dataclasses

import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N
from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict
from cosmos_predict2.net_config import CROSS_VIEW_MAP_7, DIT_2B_MULTIVIEW_CROSSVIEW, tiny_dit
from oracle import dit as odit

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


@pytest.mark.parametrize("D,M", [(2048, 3000), (512, 77), (5120, 130)])
def test_layer_norm_affine(device, D, M):
    g = torch.Generator(device=device).manual_seed(D)
    x = (torch.randn(M, D, generator=g, device=device) * 3 + 1).to(BF16)
    w = (1 + 0.2 * torch.randn(D, generator=g, device=device)).to(BF16)
    b = (0.2 * torch.randn(D, generator=g, device=device)).to(BF16)
    got = N.layer_norm(x, w, b)
    ref = F.layer_norm(x.float(), (D,), w.float(), b.float(), eps=1e-6)
    err = (got.float() - ref).abs().max().item()
    assert err <= 2 ** -7 * ref.abs().max().item(), err  # one bf16 rounding of the fp32 result
    assert ((got.float() - ref).norm() / ref.norm()).item() <= 2e-3


def _case(device, cfg, view_ids, t_view, hp, wp, seed=4):
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=seed, zero_adaln_out=False).items()}
    V = len(view_ids)
    T = V * t_view
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, 16, T, 2 * hp, 2 * wp, generator=g)
    mask = torch.zeros(1, 1, T, 2 * hp, 2 * wp)
    mask[:, :, ::t_view] = 1
    t = torch.tensor([[0.3] * T])
    ctx = torch.randn(1, 512 * V, cfg.crossattn_proj_in_channels, generator=g).to(BF16)
    vi = torch.tensor([view_ids]).repeat_interleave(t_view, dim=1)
    net = MinimalV1LVGDiT(cfg, device=device)
    net.load_state_dict(sd)
    out = net(x.to(device).to(BF16), t.to(device), ctx.to(device), condition_video_input_mask_B_C_T_H_W=mask.to(device),
              view_indices_B_T=vi.to(device))
    torch.cuda.synchronize()
    sd_dev = {k: v.to(device) for k, v in sd.items()}
    ref = odit.dit_forward(dataclasses.asdict(cfg), sd_dev, x.to(device), t.to(device), ctx.to(device), mask.to(device),
                           view_ids=view_ids)
    return ((out.float() - ref.float()).norm() / ref.float().norm()).item(), out


@pytest.mark.parametrize("wan_fp32", [False, True])
@pytest.mark.parametrize("view_ids", [[0, 1, 2], [0, 2], [2, 1]])
def test_crossview_tiny_matches_oracle(device, view_ids, wan_fp32):
    """wan_fp32=False: the registered cross-view net's bf16 conditioning (defaults/net.py:105); True: the fp32
    strategy on the same layout."""
    cfg = tiny_dit(num_blocks=2, n_cameras_emb=3, state_t=2, adaln_view_embedding=True,
                   cross_view_attn_map=((1, 2), (0,), (0, 1)), use_wan_fp32_strategy=wan_fp32)
    rel, out = _case(device, cfg, view_ids, 2, 4, 8)
    print(f"cross-view tiny net, views {view_ids}, wan_fp32 {wan_fp32}: rel-L2 {rel:.3e}")
    assert torch.isfinite(out).all() and rel <= 1e-2, rel


def test_crossview_2b_width_seven_views(device):
    """The registered 2B cross-view net's widths and 7-view neighbour map (one block), 7 views x 8 latent frames of
    16 x 26 tokens (23 296 tokens, CFG-sized batch 1)."""
    cfg = dataclasses.replace(DIT_2B_MULTIVIEW_CROSSVIEW, num_blocks=1)
    assert cfg.cross_view_attn_map == CROSS_VIEW_MAP_7 and not cfg.use_wan_fp32_strategy
    rel, out = _case(device, cfg, list(range(7)), 8, 16, 26)
    print(f"cross-view 2B-width block, 7 views: rel-L2 {rel:.3e}")
    assert torch.isfinite(out).all() and rel <= 1e-2, rel
