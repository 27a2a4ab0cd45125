"""Inference API: the reference's cosmos_predict2/inference.py (Inference(SetupArguments).generate).

Inference(args).generate(samples, output_dir) -> list of written paths. Videos are written as .mp4
at 16 fps like the reference (inference.py:151-171, imaginaire/visualize/video.py), by this build's
own H.264 I_PCM muxer (video_io.py: no ffmpeg ships in this image). Guardrails and
the Reason1 text encoder are outside this build: prompt embeddings come from the
pipeline's `text_encoder` callable.
"""
from __future__ import annotations

import logging
from pathlib import Path
from typing import List, Optional

import numpy as np
import torch

from .config import InferenceArguments, SetupArguments, is_rank0, path_to_str
from .pipeline import Video2WorldInference
from .video_io import write_mp4

log = logging.getLogger("cosmos_predict2")


def save_video(video_0_1_C_T_H_W: torch.Tensor, path_stem: str, fps: int = 16) -> str:
    """[C, T, H, W] in [0, 1] -> <stem>.mp4 (uint8 frames, as save_img_or_video does)."""
    frames = (video_0_1_C_T_H_W * 255.0).clamp(0, 255).to(torch.uint8).permute(1, 2, 3, 0).cpu().numpy()
    return write_mp4(np.ascontiguousarray(frames), path_stem + ".mp4", fps=fps)


class Inference:
    def __init__(self, args: SetupArguments, text_encoder=None):
        torch.set_grad_enabled(False)
        self.setup_args = args
        self.rank0 = is_rank0()
        self.pipe = Video2WorldInference(args.model, ckpt_path=args.checkpoint_path, tokenizer_path=args.tokenizer_path,
                                         context_parallel_size=args.context_parallel_size or 1,
                                         state_t=args.state_t, text_encoder=text_encoder)
        if self.rank0:
            Path(args.output_dir).mkdir(parents=True, exist_ok=True)

    def generate(self, samples: List[InferenceArguments], output_dir: Path) -> List[str]:
        out: List[str] = []
        for s in samples:
            p = self._generate_sample(s, Path(output_dir))
            if p is not None:
                out.append(p)
        return out

    def _generate_sample(self, sample: InferenceArguments, output_dir: Path) -> Optional[str]:
        stem = output_dir / sample.name
        if self.rank0:
            output_dir.mkdir(parents=True, exist_ok=True)
            (Path(str(stem) + ".json")).write_text(sample.model_dump_json())
        try:
            if sample.enable_autoregressive:
                video = self.pipe.generate_autoregressive_from_batch(
                    prompt=sample.prompt, input_path=path_to_str(sample.input_path),
                    num_output_frames=sample.num_output_frames, chunk_size=sample.chunk_size,
                    chunk_overlap=sample.chunk_overlap, guidance=sample.guidance,
                    num_latent_conditional_frames=sample.num_input_frames, resolution=sample.resolution,
                    seed=sample.seed, negative_prompt=sample.negative_prompt, num_steps=sample.num_steps)
            else:
                video = self.pipe.generate_vid2world(
                    prompt=sample.prompt, input_path=path_to_str(sample.input_path), guidance=sample.guidance,
                    num_video_frames=sample.num_output_frames, num_latent_conditional_frames=sample.num_input_frames,
                    resolution=sample.resolution, seed=sample.seed, negative_prompt=sample.negative_prompt,
                    num_steps=sample.num_steps)
        except Exception:
            if self.setup_args.keep_going:
                log.exception("sample %s failed", sample.name)
                return None
            raise
        if self.rank0:
            return save_video((1.0 + video[0]) / 2, str(stem))
        return str(stem) + ".mp4"
