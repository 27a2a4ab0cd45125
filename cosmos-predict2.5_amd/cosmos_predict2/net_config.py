"""Network / sampler hyper-parameters of the Cosmos-Predict2.5 checkpoints this build serves.

Values follow the reference's registered configs:
  * net: COSMOS_V1_2B_NET_MININET / COSMOS_V1_14B_NET_MININET
    (cosmos_predict2/_src/predict2/configs/video2world/defaults/net.py:58-94) with the rectified-flow
    experiment overrides (configs/video2world/experiment/reason_embeddings/
    model_2B_reason_1p1_rectified_flow.py:300-338, model_14b_reason_1p1_rectified_flow.py:322-344);
  * sampler: Stage-c_pt_4-Index-2-Size-2B-Res-720-Fps-16-Note-rf_with_edm_ckpt
    (configs/video2world/experiment/specialized_model/SFT_2B_RF.py:752-768: Karras sigmas,
    conditional_frame_timestep 0.1) for 2B post-trained; shift-5 linspace for the pre-trained models.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass(frozen=True)
class DiTConfig:
    model_channels: int = 2048
    num_heads: int = 16
    num_blocks: int = 28
    mlp_ratio: float = 4.0
    in_channels: int = 16  # latent channels (MinimalV1LVGDiT adds +1 for the condition mask)
    out_channels: int = 16
    patch_spatial: int = 2
    patch_temporal: int = 1
    concat_padding_mask: bool = True
    crossattn_emb_channels: int = 1024
    use_crossattn_projection: bool = True
    crossattn_proj_in_channels: int = 100352
    adaln_lora_dim: int = 256
    max_img_h: int = 240
    max_img_w: int = 240
    max_frames: int = 128
    rope_h_extrapolation_ratio: float = 3.0
    rope_w_extrapolation_ratio: float = 3.0
    rope_t_extrapolation_ratio: float = 1.0
    rope_enable_fps_modulation: bool = False
    timestep_scale: float = 0.001
    use_wan_fp32_strategy: bool = True
    # action conditioning (cosmos_predict2/_src/predict2/action/networks/action_conditioned_minimal_v1_lvg_dit.py):
    # action_dim > 0 adds action_embedder_B_D / _B_3D (Linear-GELU(tanh)-Linear MLPs) whose outputs are
    # added to the timestep embedding and the AdaLN-LoRA term before t_embedding_norm.
    action_dim: int = 0
    # > 0: ActionChunkConditionedMinimalV1LVGDiT (:182-346): actions grouped per latent frame
    # (temporal_compression_ratio of them), latent frame 0 gets a zero embedding;
    # 0: ActionConditionedMinimalV1LVGDiT (:48-179): one embedding of the whole chunk for every frame
    action_per_latent_frame: int = 0
    num_action_per_chunk: int = 12
    action_hidden: int = 0  # hidden width of the embedder MLPs (0 = 4 * model_channels)
    # multi-view (cosmos_predict2/_src/predict2_multiview/networks/multiview_dit.py:268-325): n_cameras_emb > 0
    # adds view_embeddings (nn.Embedding(n_cameras_emb, view_condition_dim)) concatenated to the input
    # channels of every view (concat_view_embedding); views are stacked along T (state_t latent frames
    # each), self-attention runs over all views jointly, RoPE positions restart per view
    # (MultiCameraVideoRopePosition3DEmb :103-130), cross-attention is per view (512 text tokens each, :40-55)
    n_cameras_emb: int = 0
    view_condition_dim: int = 0
    state_t: int = 0
    # cross-view multi-view net (MultiViewCrossDiT, predict2_multiview/networks/multiview_cross_dit.py:502-869):
    # adaln_view_embedding adds adaln_view_embedder (nn.Embedding(n_cameras_emb, D)) + adaln_view_proj (Linear(D, 9D))
    # whose 9 chunks are added to every block's shift / scale / gate per view (:355-404); a non-empty
    # cross_view_attn_map (neighbour view ids per view id) enables per-view self-attention plus a CrossViewAttention
    # sub-layer after it (:115-228, 436-450): per latent frame, each view's tokens attend to its neighbours' tokens of
    # the same frame, un-gated residual after an affine LayerNorm
    adaln_view_embedding: bool = False
    cross_view_attn_map: tuple = ()

    @property
    def head_dim(self) -> int:
        return self.model_channels // self.num_heads

    @property
    def patch_features(self) -> int:
        # (in_channels + cond mask + padding mask) * p_t * p_s * p_s
        return ((self.in_channels + 1 + int(self.concat_padding_mask) + self.view_condition_dim)
                * self.patch_temporal * self.patch_spatial ** 2)

    @property
    def mlp_hidden(self) -> int:
        return int(self.model_channels * self.mlp_ratio)

    @property
    def action_in_features(self) -> int:
        per = self.action_per_latent_frame or self.num_action_per_chunk
        return self.action_dim * per

    @property
    def action_hidden_features(self) -> int:
        return self.action_hidden or 4 * self.model_channels

    def replace(self, **kw) -> "DiTConfig":
        return dataclasses.replace(self, **kw)


@dataclass(frozen=True)
class SamplerConfig:
    """Text2WorldModelRectifiedFlowConfig / Video2WorldModelRectifiedFlowConfig fields used at inference."""

    state_ch: int = 16
    state_t: int = 24
    shift: float = 5.0
    use_kerras_sigma_at_inference: bool = False
    conditional_frame_timestep: float = -1.0
    denoise_replace_gt_frames: bool = True
    cfg_mode: str = "video2world"  # "video2world": c + g(c-u) ; "text2world": u + g(c-u)
    resolution: str = "720"


DIT_2B = DiTConfig()
DIT_14B = DiTConfig(model_channels=5120, num_heads=40, num_blocks=36)

SAMPLER_2B_POST_TRAINED = SamplerConfig(use_kerras_sigma_at_inference=True, conditional_frame_timestep=0.1)
SAMPLER_PRE_TRAINED = SamplerConfig()
# robot/action-cond (checkpoint_db.py:469-492, experiment ..._action_conditioned_rectified_flow_bridge_13frame_256x320,
# exp_2B_action_conditioned_rectify_flow.py:617-657): ActionChunk net, action_dim 7, 4 actions per latent
# frame, state_t = 1 + 12 // 4 = 4 (13 frames at 256x320), shift-5 linspace schedule, no conditional-frame
# timestep; the 2B net's rope / timestep / crossattn overrides of the base rectified-flow experiment
# (:308-320) apply on top of the /net group default.
DIT_2B_ACTION = DIT_2B.replace(action_dim=7, action_per_latent_frame=4)
SAMPLER_ACTION = SamplerConfig(state_t=4, resolution="256")
# auto/multiview (checkpoint_db.py:397-415, experiment buttercup_predict2p5_2b_7views_res720p_fps30_t8_..._nofps,
# predict2_multiview/configs/vid2vid/experiment/buttercup/buttercup2p5_rectified_flow.py:30-75, 529-550;
# net COSMOS_V1_2B_MULTIVIEW_NET, defaults/net.py:26-63): 7 camera embeddings of 7 channels, state_t 8 per
# view (29 frames), RoPE h/w 3.0, t 8/24, fps modulation off; CFG uncond + g (cond - uncond)
# (multiview_vid2vid_model_rectified_flow.py:381); the first n latent frames of every view are conditioned.
# Both multi-view nets set use_wan_fp32_strategy=False (defaults/net.py:52, 105): the t-embedding, AdaLN and final
# layer run in the net's bf16 (MinimalV1LVGDiT._time_modulation_bf16, scale_timesteps).
DIT_2B_MULTIVIEW = DIT_2B.replace(n_cameras_emb=7, view_condition_dim=7, state_t=8,
                                  rope_t_extrapolation_ratio=8.0 / 24.0, use_wan_fp32_strategy=False)
SAMPLER_MULTIVIEW = SamplerConfig(state_t=8, cfg_mode="text2world", resolution="720")
# cross-view multi-view net (COSMOS_V1_2B_MULTIVIEW_CROSSVIEW_NET, predict2_multiview/configs/vid2vid/defaults/net.py:
# 76-107: adaln view embedding, no view-embedding input channels, cross-view attention) with the crossview experiment's
# neighbour map (experiment/buttercup/buttercup2p5_rectified_flow.py:387-399) in the view ids of
# predict2_multiview/scripts/inference.py:61-69 (front_wide 0, cross_right 1, rear_right 2, rear_tele 3, rear_left 4,
# cross_left 5, front_tele 6); state_t, RoPE and use_wan_fp32_strategy=False as the multiview net above.
CROSS_VIEW_MAP_7 = ((5, 1, 6), (0, 2), (1, 3), (4, 2), (5, 3), (0, 4), (0,))
DIT_2B_MULTIVIEW_CROSSVIEW = DIT_2B.replace(n_cameras_emb=7, view_condition_dim=0, state_t=8,
                                            rope_t_extrapolation_ratio=8.0 / 24.0, adaln_view_embedding=True,
                                            cross_view_attn_map=CROSS_VIEW_MAP_7, use_wan_fp32_strategy=False)

# model name (cosmos_predict2/config.py ModelKey.name) -> (net, sampler)
MODELS = {
    "2B/post-trained": (DIT_2B, SAMPLER_2B_POST_TRAINED),
    "2B/pre-trained": (DIT_2B, SAMPLER_PRE_TRAINED),
    "14B/pre-trained": (DIT_14B, SAMPLER_PRE_TRAINED),
    "2B/robot/action-cond": (DIT_2B_ACTION, SAMPLER_ACTION),
    "2B/auto/multiview": (DIT_2B_MULTIVIEW, SAMPLER_MULTIVIEW),
    # the reference registers this net (hydra net "cosmos_v1_2B_multiview_crossview") but ships no checkpoint for it
    "2B/auto/multiview-crossview": (DIT_2B_MULTIVIEW_CROSSVIEW, SAMPLER_MULTIVIEW),
}

# Subset of VIDEO_RES_SIZE_INFO (cosmos_predict2/_src/predict2/datasets/utils.py:44-67); the model's
# default resolution is the "9,16" entry read as (H, W) (text2world_model_rectified_flow.py:872-873).
VIDEO_RES_SIZE_INFO = {
    "720": {"1,1": (960, 960), "4,3": (960, 704), "3,4": (704, 960), "16,9": (1280, 704), "9,16": (704, 1280)},
    "480": {"1,1": (480, 480), "4,3": (640, 480), "3,4": (480, 640), "16,9": (768, 432), "9,16": (432, 768)},
    "256": {"1,1": (256, 256), "4,3": (320, 256), "3,4": (256, 320), "16,9": (320, 192), "9,16": (192, 320)},
}


def tiny_dit(**kw) -> DiTConfig:
    """A small configuration with the 2B layout for tests (head dim 128)."""
    base = DiTConfig(model_channels=512, num_heads=4, num_blocks=2, crossattn_emb_channels=256,
                     crossattn_proj_in_channels=384, adaln_lora_dim=64)
    return base.replace(**kw)
