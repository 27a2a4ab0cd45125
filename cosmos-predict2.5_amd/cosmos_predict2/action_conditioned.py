"""Action-conditioned autoregressive video generation (robot/action-cond model) on MI355X.

Mirrors the reference's cosmos_predict2/action_conditioned.py (inference loop :205-380, action
extraction :44-135) and the rotation helpers it uses (_src/predict2/action/datasets/dataset_utils.py:
108-140, 153-182, 220-251): robot states -> relative end-effector actions (scaled), then a sliding
chunk loop in which every chunk of `chunk_size` actions generates chunk_size + 1 frames conditioned on
the previous chunk's last frame (re-quantised to uint8), seed = the chunk's first action index.
The network is the ActionChunk DiT (dit.MinimalV1LVGDiT with DiTConfig.action_dim > 0); context
parallelism, the HIP kernels and the sampler are those of the Image2World path.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from .pipeline import DEFAULT_NEGATIVE_PROMPT, Video2WorldInference


# ----------------------------------------------------------------------------- rotations (ZYX Euler)
def _rx(a):
    return np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])


def _ry(b):
    return np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])


def _rz(c):
    return np.array([[np.cos(c), -np.sin(c), 0], [np.sin(c), np.cos(c), 0], [0, 0, 1]])


def euler2rotm(euler) -> np.ndarray:
    """(roll, pitch, yaw) -> R = Rz(yaw) Ry(pitch) Rx(roll) (dataset_utils.py:128-140)."""
    return _rz(euler[2]) @ _ry(euler[1]) @ _rx(euler[0])


def _wrap(a: float) -> float:
    while a > np.pi:
        a -= 2 * np.pi
    while a <= -np.pi:
        a += 2 * np.pi
    return a


def rotm2euler(R) -> np.ndarray:
    """Inverse of euler2rotm, angles in (-pi, pi] (dataset_utils.py:153-182)."""
    R = np.asarray(R, dtype=float)
    if np.linalg.norm(np.identity(3) - R.T @ R) >= 1e-6:
        raise ValueError("not a rotation matrix")
    sy = math.sqrt(R[0, 0] ** 2 + R[1, 0] ** 2)
    if sy >= 1e-6:
        x, y, z = math.atan2(R[2, 1], R[2, 2]), math.atan2(-R[2, 0], sy), math.atan2(R[1, 0], R[0, 0])
    else:
        x, y, z = math.atan2(-R[1, 2], R[1, 1]), math.atan2(-R[2, 0], sy), 0.0
    return np.array([_wrap(x), _wrap(y), _wrap(z)])


def rotm2quat(R) -> np.ndarray:
    """Rotation matrix -> quaternion (w, x, y, z), largest-diagonal branch (dataset_utils.py:220-251)."""
    R = np.asarray(R, dtype=float)
    tr = np.trace(R)
    if tr > 0:
        s = 0.5 / np.sqrt(tr + 1.0)
        return np.array([0.25 / s, (R[2, 1] - R[1, 2]) * s, (R[0, 2] - R[2, 0]) * s, (R[1, 0] - R[0, 1]) * s])
    if R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2])
        return np.array([(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s])
    if R[1, 1] > R[2, 2]:
        s = 2.0 * np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2])
        return np.array([(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s])
    s = 2.0 * np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1])
    return np.array([(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s])


# ----------------------------------------------------------------------------- actions
def relative_actions(arm_states: np.ndarray, gripper_states: np.ndarray, use_quat: bool = False) -> np.ndarray:
    """[L, 6] (xyz, rpy) + [L] gripper -> [L-1, 7 | 8]: end-effector motion in the previous frame's
    coordinates [rel_xyz, rel_rot (Euler or quaternion), next gripper] (action_conditioned.py:62-104)."""
    L = len(arm_states)
    out = np.zeros((L - 1, 8 if use_quat else 7))
    for k in range(1, L):
        prev_r = euler2rotm(arm_states[k - 1, 3:6])
        cur_r = euler2rotm(arm_states[k, 3:6])
        rel_xyz = prev_r.T @ (arm_states[k, 0:3] - arm_states[k - 1, 0:3])
        rel = prev_r.T @ cur_r
        rot = rotm2quat(rel) if use_quat else rotm2euler(rel)
        out[k - 1, 0:3] = rel_xyz
        out[k - 1, 3:3 + len(rot)] = rot
        out[k - 1, -1] = gripper_states[k]
    return out


def get_action_sequence_from_states(data: dict, fps_downsample_ratio: int = 1, use_quat: bool = False,
                                    state_key: str = "state", gripper_scale: float = 1.0,
                                    gripper_key: str = "continuous_gripper_state",
                                    action_scaler: float = 20.0) -> np.ndarray:
    """Annotation dict -> scaled action sequence (action_conditioned.py:107-135)."""
    arm = np.array(data[state_key])[::fps_downsample_ratio]
    grip = np.array(data[gripper_key])[::fps_downsample_ratio]
    act = relative_actions(arm, grip, use_quat=use_quat)
    if use_quat:  # the reference's scale vector has 7 entries; its quaternion path is not scaled there
        raise NotImplementedError("use_quat=True: the reference scales a 7-wide action (action_conditioned.py:130)")
    return act * np.array([action_scaler] * 6 + [gripper_scale])


# ----------------------------------------------------------------------------- generation loop
def conditioning_video(img: np.ndarray, n_frames: int) -> torch.Tensor:
    """uint8 [1, 3, n_frames, H, W]: frame 0 the uint8 image [H, W, 3], the rest zeros. The reference
    (cosmos_predict2/action_conditioned.py:326-331) builds it as to_tensor (fp32 / 255), zero frames, then
    `(vid * 255.0).to(torch.uint8)`; that fp32 round trip returns every uint8 value unchanged, so the uint8 frame is
    used directly (no fp32 video on the host: ~30 ms per chunk at 480x640)."""
    H, W, _ = img.shape
    vid = torch.zeros(1, 3, n_frames, H, W, dtype=torch.uint8)
    vid[0, :, 0] = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)
    return vid


class ActionConditionedInference:
    """The reference's action-conditioned `inference()` chunk loop over one trajectory."""

    def __init__(self, pipe: Optional[Video2WorldInference] = None, **pipe_kwargs):
        self.pipe = pipe or Video2WorldInference("2B/robot/action-cond", **pipe_kwargs)

    @torch.no_grad()
    def generate(self, initial_frame: np.ndarray, actions: np.ndarray, chunk_size: int = 12, guidance: float = 7,
                 num_latent_conditional_frames: int = 1, prompt: str = "", start_frame_idx: int = 0,
                 negative_prompt: str = DEFAULT_NEGATIVE_PROMPT, num_steps: int = 35, single_chunk: bool = False,
                 max_frames: Optional[int] = None) -> np.ndarray:
        """initial_frame uint8 [H, W, 3] (already at the model resolution), actions [N, action_dim]
        -> uint8 video [T, H, W, 3] (first chunk whole, later chunks' first chunk_size frames,
        action_conditioned.py:291-366). max_frames stops once that many frames exist."""
        H, W, _ = initial_frame.shape
        img = initial_frame
        chunks = []
        total = 0
        for i in range(start_frame_idx, len(actions), chunk_size):
            a = actions[i:i + chunk_size]
            if a.shape[0] != chunk_size:  # zero-pad an incomplete last chunk
                a = np.concatenate([a, np.zeros((chunk_size - a.shape[0],) + a.shape[1:], a.dtype)], 0)
            n_frames = chunk_size + 1
            # the reference's to_tensor (/ 255) -> zero frames -> * 255 -> uint8 round trip is the identity on every
            # uint8 value in fp32 (tests/test_action_cpu.py), so the uint8 frame goes in as it is: [1, C, T, H, W]
            vid = conditioning_video(img, n_frames)
            video = self.pipe.generate_vid2world(prompt, vid, guidance=guidance, num_video_frames=n_frames,
                                                 num_latent_conditional_frames=num_latent_conditional_frames,
                                                 resolution=f"{H},{W}", seed=i, negative_prompt=negative_prompt,
                                                 num_steps=num_steps, action=torch.from_numpy(a).float())
            v = ((torch.clamp((video + 1) / 2, 0, 1)[0] * 255).to(torch.uint8).permute(1, 2, 3, 0).cpu().numpy())
            img = v[-1]
            chunks.append(v if not chunks else v[:chunk_size])
            total += len(chunks[-1])
            if single_chunk or (max_frames is not None and total >= max_frames):
                break
        out = np.concatenate(chunks, 0)
        return out[:max_frames] if max_frames is not None else out
