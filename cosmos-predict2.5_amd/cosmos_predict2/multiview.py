"""Multi-view (auto/multiview) video generation on MI355X.

Mirrors the reference's multi-view inference: cosmos_predict2/multiview.py (MultiviewInference) over
_src/predict2_multiview/scripts/inference.py:166-230 (Vid2VidInference.generate_from_batch) and
_src/predict2_multiview/models/multiview_vid2vid_model_rectified_flow.py (per-view VAE encode/decode
:69-91, per-view text context :420-534, CFG uncond + g (cond - uncond) :381). V camera views are
stacked along the latent T axis (V x state_t frames); the network is dit.MinimalV1LVGDiT with
DiTConfig.n_cameras_emb > 0 (view-embedding input channels, per-view RoPE and cross-attention, joint
self-attention over all views), sampled by the same fused UniPC/CFG loop and context-parallel
token sharding as Image2World.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import torch

from .pipeline import Video2WorldInference

# view order of the driving rig (predict2_multiview/datasets/local_dataset.py:18-26)
VIEW_INDEX_DICT = {"front_wide": 0, "cross_right": 1, "rear_right": 2, "rear": 3, "rear_left": 4,
                   "cross_left": 5, "front_tele": 6}


class MultiviewInference:
    """`generate(views, prompt, ...)` -> [1, 3, V*T, H, W] (stack_mode "time") or [1, 3, T, V*H, W]."""

    def __init__(self, pipe: Optional[Video2WorldInference] = None, **pipe_kwargs):
        pipe_kwargs.setdefault("model_name", "2B/auto/multiview")
        self.pipe = pipe or Video2WorldInference(**pipe_kwargs)

    def _text_context(self, prompt: Union[str, Sequence[str]], n_views: int, front: int = 0) -> torch.Tensor:
        """[1, V*512, E]: one caption -> the front camera's 512 tokens, the empty string's elsewhere
        (compute_text_embeddings_online_multiview_single_caption :420-457); V captions (a list or
        " -- "-joined) -> one 512-token block per view (:460-514)."""
        enc = self.pipe.text_encoder
        caps = list(prompt) if not isinstance(prompt, str) else prompt.split(" -- ")
        if len(caps) == 1:
            blocks = [enc("") for _ in range(n_views)]
            blocks[front] = enc(caps[0])
        elif len(caps) == n_views:
            blocks = [enc(c) for c in caps]
        else:
            raise ValueError(f"Expected 1 or {n_views} captions, got {len(caps)}")
        return torch.cat([b.to(self.pipe.device) for b in blocks], 1)

    @torch.no_grad()
    def generate(self, views: List[Optional[torch.Tensor]], prompt: Union[str, Sequence[str]],
                 num_conditional_frames: int = 1, guidance: float = 7, seed: int = 1, num_steps: int = 35,
                 stack_mode: str = "time", resolution: Optional[str] = None,
                 view_indices: Optional[Sequence[int]] = None) -> torch.Tensor:
        """views: per camera a uint8 video [3, T_pix, H, W] (None = no input for that view: text2world);
        T_pix = tokenizer.get_pixel_num_frames(state_t). Returns fp32 video in [-1, 1]."""
        model = self.pipe.model
        tok = model.tokenizer
        st = model.net.cfg.state_t or model.config.state_t
        V = len(views)
        t_pix = tok.get_pixel_num_frames(st)
        if resolution is not None:
            H, W = (int(x) for x in resolution.split(","))
        else:
            ref = next((v for v in views if v is not None), None)
            if ref is None:
                raise ValueError("give `resolution` when no view has an input video")
            H, W = ref.shape[-2:]
        sc = tok.spatial_compression_factor
        h, w = H // sc, W // sc
        gt = None
        if num_conditional_frames > 0:
            lat = []
            for v in views:  # per-view encode (multiview_vid2vid_model_rectified_flow.py:69-79)
                vid = torch.zeros(1, 3, t_pix, H, W, dtype=torch.uint8) if v is None else v[None]
                lat.append(model.encode_conditioning(vid, num_conditional_frames, st))
            gt = torch.cat(lat, 2)
        ctx_c = self._text_context(prompt, V)
        ctx_u = torch.zeros_like(ctx_c)  # is_negative_prompt=False: text dropout embedding (scripts/inference.py:186)
        vi = None if view_indices is None else torch.tensor(list(view_indices), device=self.pipe.device)
        latents = model.sample_latents(gt, ctx_c, ctx_u, state_shape=(model.config.state_ch, V * st, h, w),
                                       num_conditional_frames=num_conditional_frames, guidance=guidance, seed=seed,
                                       num_steps=num_steps, view_indices=vi)
        video = torch.cat([model.decode(latents[:, :, i * st:(i + 1) * st]).float() for i in range(V)], 2)
        if stack_mode == "height":  # b c (v t) h w -> b c t (v h) w (scripts/inference.py:224-225)
            B, C, VT, Hh, Ww = video.shape
            video = video.view(B, C, V, VT // V, Hh, Ww).permute(0, 1, 3, 2, 4, 5).reshape(B, C, VT // V, V * Hh, Ww)
        elif stack_mode != "time":
            raise ValueError(f"Invalid stack mode '{stack_mode}'. Must be one of: {{'height', 'time'}}")
        return video
