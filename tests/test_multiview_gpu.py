"""Multi-view generation on the device (tiny multi-view net, Wan VAE layout with seeded weights):
per-view encode of the conditioning frames, V views stacked on the latent T axis, per-view decode
(predict2_multiview scripts/inference.py:166-230)."""
import pytest
import torch

from cosmos_predict2.multiview import MultiviewInference
from cosmos_predict2.net_config import CROSS_VIEW_MAP_7, SamplerConfig, tiny_dit
from cosmos_predict2.pipeline import Video2WorldInference

pytestmark = pytest.mark.gpu


def test_multiview_generate_shapes_and_conditioning(device):
    cfg = tiny_dit(num_blocks=1, n_cameras_emb=7, view_condition_dim=7, state_t=2, use_wan_fp32_strategy=False)
    pipe = Video2WorldInference("2B/auto/multiview", device=device, net_cfg=cfg,
                                sampler_cfg=SamplerConfig(state_t=2, cfg_mode="text2world"))
    mv = MultiviewInference(pipe)
    g = torch.Generator().manual_seed(0)
    views = [torch.randint(0, 256, (3, 5, 64, 80), generator=g, dtype=torch.uint8) for _ in range(3)]
    v = mv.generate(views, "a car drives down a street", num_conditional_frames=1, num_steps=2, seed=3)
    assert v.shape == (1, 3, 15, 64, 80) and torch.isfinite(v).all()
    vh = mv.generate(views, "a car drives down a street", num_conditional_frames=1, num_steps=2, seed=3,
                     stack_mode="height")
    assert vh.shape == (1, 3, 5, 192, 80)
    assert torch.equal(vh[:, :, :, 64:128], v[:, :, 5:10])  # view 1 stacked under view 0
    t2w = mv.generate([None, None], "x -- y", num_conditional_frames=0, num_steps=2, resolution="64,80")
    assert t2w.shape == (1, 3, 10, 64, 80)


def test_crossview_generate(device):
    """The cross-view net (MultiViewCrossDiT) through the same multi-view pipeline: 3 of the 7 rig views (ids 0, 1, 2:
    front_wide, cross_right, rear_right, so rear_right's neighbour rear_tele is absent and masked out)."""
    cfg = tiny_dit(num_blocks=1, n_cameras_emb=7, state_t=2, adaln_view_embedding=True, use_wan_fp32_strategy=False,
                   cross_view_attn_map=CROSS_VIEW_MAP_7)
    pipe = Video2WorldInference("2B/auto/multiview-crossview", device=device, net_cfg=cfg,
                                sampler_cfg=SamplerConfig(state_t=2, cfg_mode="text2world"))
    mv = MultiviewInference(pipe)
    g = torch.Generator().manual_seed(0)
    views = [torch.randint(0, 256, (3, 5, 64, 80), generator=g, dtype=torch.uint8) for _ in range(3)]
    v = mv.generate(views, "a car drives down a street", num_conditional_frames=1, num_steps=2, seed=3)
    assert v.shape == (1, 3, 15, 64, 80) and torch.isfinite(v).all()
