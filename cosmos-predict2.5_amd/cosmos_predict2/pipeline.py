"""Video2WorldInference: input processing, data batch, sampling, decode (MI355X build).

Mirrors cosmos_predict2/_src/predict2/inference/video2world.py:
  resize_input :75-97, read_and_process_image :100-142, read_and_process_video :145-233 (frames given
  as a uint8 tensor here: no mp4 demuxer ships in this image), Video2WorldInference :236-820
  (_get_data_batch_input :317-383, generate_vid2world :385-580, generate_autoregressive_from_batch
  :582-810).
The Reason1 text encoder is outside the hot path: prompts are turned into
[1, 512, 100352] embeddings by a pluggable `text_encoder` callable; the default one loads
precomputed embeddings (torch.load(weights_only=True)) or, for benchmarking, derives seeded N(0, 1)
embeddings from the prompt (`synthetic_text_encoder`).
"""
from __future__ import annotations

import hashlib
import math
import os
from typing import Callable, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import context_parallel as cpu
from .dit import init_state_dict
from .model import NUM_CONDITIONAL_FRAMES_KEY, Video2WorldModelRectifiedFlow
from .net_config import MODELS, VIDEO_RES_SIZE_INFO, DiTConfig, SamplerConfig
from .vae import Wan2pt1VAEInterface, init_vae_state_dict

_IMAGE_EXTENSIONS = [".png", ".jpg", ".jpeg", ".webp"]
_VIDEO_EXTENSIONS = [".mp4"]
DEFAULT_NEGATIVE_PROMPT = (
    "The video captures a series of frames showing ugly scenes, static with no motion, motion blur, "
    "over-saturation, shaky footage, low resolution, grainy texture, pixelated images, poorly lit areas, "
    "underexposed and overexposed scenes, poor color balance, washed out colors, choppy sequences, jerky "
    "movements, low frame rate, artifacting, color banding, unnatural transitions, outdated special effects, "
    "fake elements, unconvincing visuals, poorly edited content, jump cuts, visual noise, and flickering. "
    "Overall, the video is of poor quality."
)
TEXT_EMB_SHAPE = (1, 512, 100352)


def synthetic_text_encoder(prompt: str, device="cuda", dim: int = TEXT_EMB_SHAPE[2]) -> torch.Tensor:
    """Deterministic N(0, 1) embedding per prompt (matches the mean-normalized Reason1 layer stats)."""
    seed = int.from_bytes(hashlib.sha256(prompt.encode()).digest()[:4], "little")
    g = torch.Generator(device=device).manual_seed(seed)
    shape = TEXT_EMB_SHAPE[:2] + (dim,)
    return torch.randn(shape, generator=g, device=device, dtype=torch.float32).to(torch.bfloat16)


def resize_input(video: torch.Tensor, resolution) -> torch.Tensor:
    """uint8 [T, C, H, W]: resize so both sides cover the target (aspect kept), then center-crop."""
    orig_h, orig_w = video.shape[2], video.shape[3]
    th, tw = resolution
    r = max(tw / orig_w, th / orig_h)
    rh, rw = int(math.ceil(r * orig_h)), int(math.ceil(r * orig_w))
    if (rh, rw) != (orig_h, orig_w):
        v = F.interpolate(video.float(), size=(rh, rw), mode="bilinear", align_corners=False, antialias=True)
        video = v.round_().clamp_(0, 255).to(torch.uint8)
    top = int(round((rh - th) / 2.0))
    left = int(round((rw - tw) / 2.0))
    return video[:, :, top: top + th, left: left + tw]


def read_and_process_image(img_path: str, resolution, num_video_frames: int, resize: bool = True) -> torch.Tensor:
    ext = os.path.splitext(img_path)[1]
    if ext not in _IMAGE_EXTENSIONS:
        raise ValueError(f"Invalid image extension: {ext}")
    from PIL import Image

    img = np.asarray(Image.open(img_path).convert("RGB"))
    img = torch.from_numpy(img.copy()).permute(2, 0, 1)[None].float() / 255.0  # [1, 3, H, W]
    vid = torch.cat([img, torch.zeros_like(img).repeat(num_video_frames - 1, 1, 1, 1)], 0)
    vid = (vid * 255.0).to(torch.uint8)
    if resize:
        vid = resize_input(vid, resolution)
    return vid.unsqueeze(0).permute(0, 2, 1, 3, 4)  # [1, C, T, H, W]


def process_video_frames(frames_uint8_T_H_W_C: torch.Tensor, resolution, num_video_frames: int,
                         num_latent_conditional_frames: int = 2, resize: bool = True,
                         validate: bool = True) -> torch.Tensor:
    """read_and_process_video on already-decoded frames: keep the last 4(n-1)+1, pad with the last.
    validate=False: the AR loop's copy of this logic (video2world.py:657-690) accepts any n."""
    if validate and num_latent_conditional_frames not in (1, 2):
        raise ValueError(f"num_latent_conditional_frames must be 1 or 2, but got {num_latent_conditional_frames}")
    v = frames_uint8_T_H_W_C.float().permute(3, 0, 1, 2) / 255.0  # [C, T, H, W]
    need = 4 * (num_latent_conditional_frames - 1) + 1
    if v.shape[1] < need:
        raise ValueError(f"Video has only {v.shape[1]} frames but needs at least {need} frames")
    C, _, H, W = v.shape
    full = torch.zeros(C, num_video_frames, H, W)
    ext = v[:, v.shape[1] - need:]
    full[:, :need] = ext
    if need < num_video_frames:
        full[:, need:] = ext[:, -1:].repeat(1, num_video_frames - need, 1, 1)
    full = (full.permute(1, 0, 2, 3) * 255.0).to(torch.uint8)
    if resize:
        full = resize_input(full, resolution)
    return full.unsqueeze(0).permute(0, 2, 1, 3, 4)


class Video2WorldInference:
    """Pipeline object of the reference's Video2WorldInference, on the MI355X model."""

    def __init__(self, model_name: str = "2B/post-trained", ckpt_path: Optional[str] = None,
                 tokenizer_path: Optional[str] = None, context_parallel_size: int = 1, device=None,
                 state_t: Optional[int] = None, text_encoder: Optional[Callable] = None,
                 net_cfg: Optional[DiTConfig] = None, sampler_cfg: Optional[SamplerConfig] = None,
                 weights_seed: int = 0, linear_precision: str = "bf16", attention_precision: str = "bf16"):
        """linear_precision: "bf16" (the reference's arithmetic) or "fp8" (the DiT block GEMMs as fp8
        MFMA, config 5's option; MinimalV1LVGDiT.set_linear_precision). attention_precision: "bf16", "fp8qk"
        (self-attention Q K^T on e4m3) or "fp8" (also P.V; MinimalV1LVGDiT.set_attention_precision)."""
        if device is None:
            device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        self.device = torch.device(device)
        ncfg, scfg = MODELS[model_name]
        ncfg = net_cfg or ncfg
        scfg = sampler_cfg or scfg
        if state_t is not None:
            import dataclasses

            scfg = dataclasses.replace(scfg, state_t=state_t)
        self.context_parallel_size = context_parallel_size
        self.process_group = None
        if context_parallel_size > 1:
            self._init_distributed()
        # tokenizer
        if tokenizer_path is not None:
            vae_sd = torch.load(tokenizer_path, map_location="cpu", weights_only=True)
        else:
            vae_sd = init_vae_state_dict(seed=weights_seed + 1, device=self.device)
        tokenizer = Wan2pt1VAEInterface(vae_sd, device=self.device, temporal_window=16)
        del vae_sd
        self.model = Video2WorldModelRectifiedFlow(ncfg, scfg, tokenizer=tokenizer, device=self.device)
        if ckpt_path is not None:
            from .checkpoint import load_dit_checkpoint

            sd = load_dit_checkpoint(ckpt_path)
        else:
            sd = init_state_dict(ncfg, seed=weights_seed, device=self.device)
        self.model.load_state_dict(sd)
        del sd
        self.model.net.set_linear_precision(linear_precision)
        self.model.net.set_attention_precision(attention_precision)
        if self.process_group is not None:
            self.model.set_context_parallel_group(self.process_group)
        emb_dim = ncfg.crossattn_proj_in_channels if ncfg.use_crossattn_projection else ncfg.crossattn_emb_channels
        self.text_encoder = text_encoder or (lambda p: synthetic_text_encoder(p, self.device, emb_dim))
        self.batch_size = 1

    def _init_distributed(self):
        import torch.distributed as dist

        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=self.device)
        world = dist.get_world_size()
        cp = self.context_parallel_size
        if world % cp:
            raise ValueError(f"world size {world} not divisible by context_parallel_size {cp}")
        rank = dist.get_rank()
        groups = [dist.new_group(list(range(g * cp, (g + 1) * cp))) for g in range(world // cp)]
        self.process_group = groups[rank // cp]

    def _get_data_batch_input(self, video: torch.Tensor, prompt: str, num_conditional_frames: int = 1,
                              negative_prompt: str = DEFAULT_NEGATIVE_PROMPT, use_neg_prompt: bool = True,
                              action: Optional[torch.Tensor] = None):
        B, C, T, H, W = video.shape
        batch = {
            "dataset_name": "video_data",
            "video": video,
            "fps": torch.randint(16, 32, (self.batch_size,)).float(),
            "padding_mask": torch.zeros(self.batch_size, 1, H, W),
            NUM_CONDITIONAL_FRAMES_KEY: num_conditional_frames,
            "t5_text_embeddings": self.text_encoder(prompt),
        }
        if use_neg_prompt:
            batch["neg_t5_text_embeddings"] = self.text_encoder(negative_prompt)
        if action is not None:  # video2world.py:352: action.unsqueeze(0) -> [1, A, action_dim]
            batch["action"] = action.unsqueeze(0) if action.dim() == 2 else action
        for k, v in batch.items():
            if isinstance(v, torch.Tensor) and torch.is_floating_point(v):
                batch[k] = v.to(self.device, torch.bfloat16)
        return batch

    @torch.no_grad()
    def generate_vid2world(self, prompt: str, input_path=None, guidance: int = 7, num_video_frames: int = 77,
                           num_latent_conditional_frames: int = 1, resolution: str = "192,320", seed: int = 1,
                           negative_prompt: str = DEFAULT_NEGATIVE_PROMPT, num_steps: int = 35,
                           action: Optional[torch.Tensor] = None, **unused) -> torch.Tensor:
        """-> video [1, 3, T, H, W] in [-1, 1] (fp32). T = tokenizer.get_pixel_num_frames(state_t) (F5).
        action: [A, action_dim] for the action-conditioned model (video2world.py:325-352)."""
        if resolution == "none":
            h, w = VIDEO_RES_SIZE_INFO[self.model.config.resolution]["9,16"]
        else:
            h, w = (int(x) for x in resolution.split(","))
        tok = self.model.tokenizer
        frames = tok.get_pixel_num_frames(self.model.config.state_t)
        if input_path is None or num_latent_conditional_frames == 0:
            vid = torch.zeros(1, 3, frames, h, w, dtype=torch.uint8)
        elif isinstance(input_path, str):
            ext = os.path.splitext(input_path)[1].lower()
            if ext in _IMAGE_EXTENSIONS:
                vid = read_and_process_image(input_path, (h, w), frames)
            elif ext in _VIDEO_EXTENSIONS:  # read_and_process_video (video2world.py:150-233)
                from .video_io import read_mp4

                vid = process_video_frames(torch.from_numpy(read_mp4(input_path)), (h, w), frames,
                                           num_latent_conditional_frames)
            else:
                raise ValueError(f"Unsupported file extension: {ext}")
        elif isinstance(input_path, torch.Tensor):
            vid = input_path
        else:
            raise ValueError(f"Unsupported input_path type: {type(input_path)}")
        import time

        t0 = time.perf_counter()
        batch = self._get_data_batch_input(vid, prompt, num_latent_conditional_frames, negative_prompt,
                                           action=action)
        latents = self.model.generate_samples_from_batch(batch, guidance=guidance, seed=seed, is_negative_prompt=True,
                                                         num_steps=num_steps)
        torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        video = self.model.decode(latents).float()
        torch.cuda.synchronize(self.device)
        self.last_timing = {"encode_and_sample_s": t1 - t0, "decode_s": time.perf_counter() - t1}
        return video

    @torch.no_grad()
    def generate_autoregressive_from_batch(self, prompt: str, input_path, num_output_frames: int, chunk_size: int,
                                           chunk_overlap: int, guidance: int = 7,
                                           num_latent_conditional_frames: int = 1, resolution: str = "192,320",
                                           seed: int = 1, negative_prompt: str = DEFAULT_NEGATIVE_PROMPT,
                                           num_steps: int = 35, **unused) -> torch.Tensor:
        """Sliding-window long-video generation (video2world.py:582-810), byte-for-byte the reference's
        window: a running uint8 input video `current_input_video` of num_output_frames frames; chunk i
        covers frames [i*(chunk_size-overlap), +chunk_size) (zero-padded to the model's frame count),
        is generated with seed + i and `chunk_overlap` as its num_latent_conditional_frames (the
        reference passes the pixel overlap there, :761-765), and writes its frames from
        [start + cond, end) back into the running video, re-quantised by truncation
        ((v/2 + 0.5).clamp(0, 1) * 255).to(uint8) (:796-804). Output: chunk 0 whole, later chunks
        without their first `chunk_overlap` frames (:785-793)."""
        if resolution == "none":
            h, w = VIDEO_RES_SIZE_INFO[self.model.config.resolution]["9,16"]
        else:
            h, w = (int(x) for x in resolution.split(","))
        frames = self.model.tokenizer.get_pixel_num_frames(self.model.config.state_t)
        full = self._ar_input_video(input_path, num_output_frames, num_latent_conditional_frames, (h, w))
        step = chunk_size - chunk_overlap
        if step <= 0:
            raise ValueError(f"chunk_overlap {chunk_overlap} must be smaller than chunk_size {chunk_size}")
        rem = num_output_frames - chunk_size
        n_chunks = 1 if rem <= 0 else 1 + (rem + step - 1) // step
        current = full.clone()
        pieces = []
        for ci in range(n_chunks):
            start = ci * step
            end = min(start + chunk_size, num_output_frames)
            if start >= num_output_frames:
                break
            n = end - start
            chunk_in = current[:, :, start:end]
            if n < frames:
                pad = torch.zeros(chunk_in.shape[:2] + (frames - n,) + chunk_in.shape[3:], dtype=chunk_in.dtype)
                chunk_in = torch.cat([chunk_in, pad], dim=2)
            n_cond = num_latent_conditional_frames if ci == 0 else chunk_overlap
            video = self.generate_vid2world(prompt, chunk_in, guidance, frames, n_cond, resolution, seed + ci,
                                            negative_prompt, num_steps)
            video = video[:, :, :n]
            pieces.append(video if ci == 0 else video[:, :, chunk_overlap:])
            if ci < n_chunks - 1:
                v8 = ((video / 2.0 + 0.5).clamp(0.0, 1.0) * 255.0).to(torch.uint8)
                current[:, :, start + n_cond:end] = v8[:, :, n_cond:].to(current.device)
        return torch.cat(pieces, dim=2)

    @staticmethod
    def _ar_input_video(input_path, num_output_frames: int, num_latent_conditional_frames: int,
                        resolution) -> torch.Tensor:
        """The AR loop's full-length uint8 input [1, 3, num_output_frames, H, W] (video2world.py:637-708):
        zeros (no input / text2world), image as frame 0 + zeros, the last 4(n-1)+1 video frames + repeats
        of the last, or a given uint8 tensor zero-padded in time."""
        h, w = resolution
        if input_path is None or num_latent_conditional_frames == 0:
            return torch.zeros(1, 3, num_output_frames, h, w, dtype=torch.uint8)
        if isinstance(input_path, torch.Tensor):
            v = input_path
            if v.shape[2] < num_output_frames:
                pad = torch.zeros(v.shape[:2] + (num_output_frames - v.shape[2],) + v.shape[3:], dtype=v.dtype)
                v = torch.cat([v, pad], dim=2)
            return v
        if not isinstance(input_path, str):
            raise ValueError(f"Unsupported input_path type: {type(input_path)}")
        ext = os.path.splitext(input_path)[1].lower()
        if ext in _IMAGE_EXTENSIONS:
            from PIL import Image

            img = np.asarray(Image.open(input_path).convert("RGB"))
            img = (torch.from_numpy(img.copy()).permute(2, 0, 1)[None].float() / 255.0 * 255.0).to(torch.uint8)
            img = resize_input(img, resolution)
            vid = torch.cat([img, torch.zeros_like(img).repeat(num_output_frames - 1, 1, 1, 1)], dim=0)
            return vid.unsqueeze(0).permute(0, 2, 1, 3, 4)
        if ext in _VIDEO_EXTENSIONS:
            from .video_io import read_mp4

            return process_video_frames(torch.from_numpy(read_mp4(input_path)), resolution, num_output_frames,
                                        num_latent_conditional_frames, validate=False)
        raise ValueError(f"Unsupported file extension: {ext}")
