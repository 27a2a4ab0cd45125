"""Sampling-loop restatement (CPU) — TEST INFRASTRUCTURE (see oracle/__init__.py).

Follows, in cosmos_predict2/_src/:
  imaginaire/utils/misc.py:158-179          arch_invariant_rand (numpy RandomState noise)
  predict2/configs/video2world/defaults/conditioner.py:45-143
                                             set_video_condition / edit_for_inference (frame mask)
  predict2/models/video2world_model_rectified_flow.py:77-138   denoise (frame replace, cond-frame t)
  predict2/models/video2world_model_rectified_flow.py:140-212  velocity_fn (cond + g (cond - uncond))
  predict2/models/text2world_model_rectified_flow.py:516-599   generate_samples_from_batch loop
Both CFG branches use the ground-truth frames (use_video_condition is True for the condition, and
edit_for_inference forces it True for the uncondition, conditioner.py:137-141).
"""
from __future__ import annotations

import numpy as np
import torch

from . import dit as odit
from .unipc import UniPC


def arch_invariant_rand(shape, seed: int) -> torch.Tensor:
    """misc.py:158-179 -> fp32 tensor."""
    return torch.from_numpy(np.random.RandomState(seed).standard_normal(shape).astype(np.float32))


def frame_mask(B: int, T: int, H: int, W: int, num_cond: int, dtype=torch.float32) -> torch.Tensor:
    """condition_video_input_mask_B_C_T_H_W: ones on the first num_cond latent frames (T > 1)."""
    m = torch.zeros(B, 1, T, H, W, dtype=dtype)
    if T > 1:
        m[:, :, :num_cond] += 1
    return m


def denoise(cfg_dit, sd, noise, xt, t_B_T, ctx, gt, mask, cond_frame_t: float, replace_gt: bool = True,
            dit_fn=None):
    """Video2WorldModelRectifiedFlow.denoise, one branch. dit_fn(cfg, sd, x, t, ctx, mask) defaults to
    the oracle DiT; tests may inject the device DiT to check the sampling plumbing alone."""
    C = xt.shape[1]
    m = mask.repeat(1, C, 1, 1, 1).type_as(xt)
    xt = gt.type_as(xt) * m + xt * (1 - m)
    if cond_frame_t >= 0:
        m_t = m.mean(dim=[1, 3, 4], keepdim=True)
        tc = torch.ones_like(m_t) * cond_frame_t
        t = (tc * m_t + t_B_T * (1 - m_t)).squeeze()
        t_B_T = t.unsqueeze(0) if t.ndim == 1 else t
    fn = dit_fn or odit.dit_forward
    out = fn(cfg_dit, sd, xt.to(odit.act_dtype()), t_B_T, ctx, mask.to(odit.act_dtype())).float()
    if replace_gt:
        gv = noise - gt.type_as(out)
        out = gv * m + out * (1 - m)
    return out


def generate(cfg_dit: dict, sd: dict, gt: torch.Tensor, ctx_cond: torch.Tensor, ctx_uncond: torch.Tensor, *,
             num_cond: int, guidance: float, seed: int, num_steps: int, shift: float = 5.0,
             use_karras: bool = False, cond_frame_t: float = -1.0, return_trajectory: bool = False,
             dit_fn=None):
    """generate_samples_from_batch for Video2World with CFG. gt: x0 latent [1, C, T, H, W] fp32. Runs on gt's device
    (the large-config tests run it on the GPU's own torch ops; the noise is drawn on the host as the reference does)."""
    B, C, T, H, W = gt.shape
    dev = gt.device
    noise = arch_invariant_rand((B, C, T, H, W), seed).to(dev)
    sched = UniPC(num_steps, shift=shift, use_karras=use_karras)
    mask = frame_mask(B, T, H, W, num_cond, dtype=gt.dtype).to(dev)
    x = noise
    traj = []
    for t in sched.timesteps:
        t_B_T = torch.stack([t]).unsqueeze(0).to(dev)  # [1, 1] int64
        vc = denoise(cfg_dit, sd, noise, x, t_B_T, ctx_cond, gt, mask, cond_frame_t, dit_fn=dit_fn)
        vu = denoise(cfg_dit, sd, noise, x, t_B_T, ctx_uncond, gt, mask, cond_frame_t, dit_fn=dit_fn)
        v = vc + guidance * (vc - vu)
        x = sched.step(v, t, x)  # shapes only differ by unit dims in the reference (:591-594)
        if return_trajectory:
            traj.append(x.clone())
    return (x, traj) if return_trajectory else x
