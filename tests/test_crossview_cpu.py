"""The cross-view multi-view net (MultiViewCrossDiT, predict2_multiview/networks/multiview_cross_dit.py:502-869) on the
CPU: the product's host path (dit.MinimalV1LVGDiT with cross_view_attn_map / adaln_view_embedding: per-view
self-attention, the cross-view sub-layer's neighbour gather and its un-gated residual, the per-view AdaLN terms) with
the libcp25 entry points replaced by the torch stand-ins of tests/cpu_kernels.py, against the oracle's restatement
(oracle/dit.py cross_view_attention / block_forward), tiny config, 3 views. Also the neighbour bookkeeping: with a
subset of the views present, absent neighbours drop out of the key sequence (the reference masks them) and a view
left without neighbours adds nothing. Tolerance rel-L2 <= 1e-2 (bf16 CPU GEMMs rounding in a different order; the
GPU test holds the device path to the same bar)."""
import dataclasses

import pytest
import torch

import __graft_entry__  # noqa: F401  (import paths)

T_VIEW, HP, WP = 2, 4, 8
MAP = ((1, 2), (0,), (0, 1))


def _cfg(wan_fp32=False):
    from cosmos_predict2.net_config import tiny_dit
    return tiny_dit(num_blocks=2, n_cameras_emb=3, state_t=T_VIEW, adaln_view_embedding=True, cross_view_attn_map=MAP,
                    use_wan_fp32_strategy=wan_fp32)


def _run(view_ids, wan_fp32=False):
    import cpu_kernels
    from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict
    from oracle import dit as odit

    cfg = _cfg(wan_fp32)
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=4, zero_adaln_out=False).items()}
    V = len(view_ids)
    T = V * T_VIEW
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, 16, T, 2 * HP, 2 * WP, generator=g)
    mask = torch.zeros(1, 1, T, 2 * HP, 2 * WP)
    mask[:, :, ::T_VIEW] = 1
    t = torch.tensor([[0.3] * T])
    ctx = torch.randn(1, 512 * V, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    vi = torch.tensor([view_ids]).repeat_interleave(T_VIEW, dim=1)
    ref = odit.dit_forward(dataclasses.asdict(cfg), sd, x, t, ctx, mask, view_ids=view_ids)
    with cpu_kernels.patched(), torch.no_grad():
        net = MinimalV1LVGDiT(cfg, device="cpu")
        net.load_state_dict(sd)
        out = net(x.to(torch.bfloat16), t, ctx, condition_video_input_mask_B_C_T_H_W=mask, view_indices_B_T=vi)
    return ((out.float() - ref).norm() / ref.norm()).item(), net


@pytest.mark.parametrize("view_ids,wan_fp32", [([0, 1, 2], False), ([0, 2], False), ([2, 1], False),
                                               ([0, 1, 2], True)])
def test_crossview_forward_matches_oracle_cpu(view_ids, wan_fp32):
    """wan_fp32=False is the registered cross-view net's conditioning arithmetic (bf16); True the fp32 strategy."""
    rel, _ = _run(view_ids, wan_fp32)
    print(f"cross-view net, views {view_ids}, wan_fp32 {wan_fp32}: rel-L2 {rel:.3e}")
    assert rel <= 1e-2, rel


def test_crossview_neighbours():
    from cosmos_predict2.dit import Geometry, MinimalV1LVGDiT

    net = MinimalV1LVGDiT(_cfg(), device="cpu")
    geo = Geometry(T=3 * T_VIEW, Hp=HP, Wp=WP, tok0=0, n_tok=3 * T_VIEW * HP * WP, n_views=3)
    assert net._cross_view_neighbours(geo, None) == [[2, 1], [0], [1, 0]]
    geo2 = dataclasses.replace(geo, T=2 * T_VIEW, n_tok=2 * T_VIEW * HP * WP, n_views=2)
    # input views (0, 2): view 0's neighbours (1, 2) -> only id 2 (position 1); view 2's (0, 1) -> id 0 (position 0)
    assert net._cross_view_neighbours(geo2, torch.tensor([0, 2])) == [[1], [0]]
    # input views (1, 2): view 1's only neighbour (0) is absent -> none; view 2's (0, 1) -> id 1 (position 0)
    assert net._cross_view_neighbours(geo2, torch.tensor([1, 2])) == [[], [0]]


@pytest.mark.parametrize("per_frame", [4, 0])
def test_action_net_bf16_conditioning_cpu(per_frame):
    """The bf16-conditioning path (use_wan_fp32_strategy=False) with action embeddings added per latent frame or per
    chunk (broadcast over the frames), host path with the CPU stand-ins, against the oracle's restatement."""
    import dataclasses

    import cpu_kernels
    from cosmos_predict2.dit import MinimalV1LVGDiT, init_state_dict
    from cosmos_predict2.net_config import tiny_dit
    from oracle import dit as odit

    cfg = tiny_dit(num_blocks=1, action_dim=7, action_per_latent_frame=per_frame, num_action_per_chunk=12,
                   use_wan_fp32_strategy=False)
    sd = {"net." + k: v for k, v in init_state_dict(cfg, seed=6, zero_adaln_out=False).items()}
    g = torch.Generator().manual_seed(2)
    T = 4
    x = torch.randn(1, 16, T, 8, 16, generator=g)
    mask = torch.zeros(1, 1, T, 8, 16)
    mask[:, :, :1] = 1
    t = torch.tensor([[0.1] + [700.0] * (T - 1)])
    ctx = torch.randn(1, 512, cfg.crossattn_proj_in_channels, generator=g).to(torch.bfloat16)
    act = torch.randn(1, 12, 7, generator=g)
    ref = odit.dit_forward(dataclasses.asdict(cfg), sd, x, t, ctx, mask, action=act)
    with cpu_kernels.patched(), torch.no_grad():
        net = MinimalV1LVGDiT(cfg, device="cpu")
        net.load_state_dict(sd)
        out = net(x.to(torch.bfloat16), t, ctx, condition_video_input_mask_B_C_T_H_W=mask, action=act)
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    print(f"action net, bf16 conditioning, per_frame={per_frame}: rel-L2 {rel:.3e}")
    assert rel <= 1e-2, rel
