"""AR sliding-window restatement (CPU) — TEST INFRASTRUCTURE (see oracle/__init__.py).

Follows cosmos_predict2/_src/predict2/inference/video2world.py:
  :693-706   a uint8 tensor input is zero-padded in time to num_output_frames
  :710-724   chunk count: 1 + ceil((N - chunk) / (chunk - overlap)) when N > chunk, else 1
  :732-759   running input video, chunk slice [start, end), zero padding to the model's frame count
  :761-783   num_latent_conditional_frames = the first chunk's value, then chunk_overlap; seed + i
  :785-793   chunk 0 stored whole, later chunks without their first chunk_overlap frames
  :795-804   re-quantisation by truncation ((v / 2 + 0.5).clamp(0, 1) * 255).to(uint8), written back
             into the running video at [start + cond, end) from the chunk's [cond:]
The model call is injected (`generate(chunk_uint8, num_latent_conditional_frames, seed)`), so the
window logic is checked byte-for-byte with a stand-in denoiser.
"""
from __future__ import annotations

from typing import Callable, List, Tuple

import torch


def chunk_plan(num_output_frames: int, chunk_size: int, chunk_overlap: int) -> List[Tuple[int, int]]:
    """[(start, end)] of every chunk that runs (:716-744)."""
    stride = chunk_size - chunk_overlap
    extra = num_output_frames - chunk_size
    count = 1 if extra <= 0 else 1 + -(-extra // stride)
    plan = []
    for i in range(count):
        s = i * stride
        if s >= num_output_frames:
            break
        plan.append((s, min(s + chunk_size, num_output_frames)))
    return plan


def autoregressive(generate: Callable, video_u8: torch.Tensor, num_output_frames: int, chunk_size: int,
                   chunk_overlap: int, model_frames: int, first_num_cond: int, seed: int) -> torch.Tensor:
    """-> the assembled video [1, 3, num_output_frames, H, W] (dtype of `generate`'s output)."""
    B, C, Tin, H, W = video_u8.shape
    running = torch.zeros(B, C, max(Tin, num_output_frames), H, W, dtype=torch.uint8)
    running[:, :, :Tin] = video_u8
    plan = chunk_plan(num_output_frames, chunk_size, chunk_overlap)
    out = []
    for i, (s, e) in enumerate(plan):
        inp = torch.zeros(B, C, max(model_frames, e - s), H, W, dtype=torch.uint8)
        inp[:, :, : e - s] = running[:, :, s:e]
        cond = first_num_cond if i == 0 else chunk_overlap
        gen = generate(inp, cond, seed + i)[:, :, : e - s]
        out.append(gen[:, :, (0 if i == 0 else chunk_overlap):])
        if i + 1 < len(plan):
            q = torch.clamp(gen / 2.0 + 0.5, 0.0, 1.0).mul(255.0).to(torch.uint8)
            running[:, :, s + cond:e] = q[:, :, cond:]
    return torch.cat(out, dim=2)
