"""User-facing arguments: the reference's cosmos_predict2/config.py API (pydantic models).

SetupArguments / InferenceArguments keep the reference's field names, defaults and validation
(cosmos_predict2/config.py:198-472): seed 0, guidance 7 (0..7), num_steps 35, the default negative
prompt, inference_type text2world / image2world / video2world -> 0 / 1 / 2 conditioning latent
frames, resolution "H,W" or "none". Checkpoint selection maps a model name to local files (no Hugging
Face download in this build: `checkpoint_path` / `tokenizer_path` point at local files, or are left
None for seeded synthetic weights).
"""
from __future__ import annotations

import enum
import json
import os
from functools import cached_property
from pathlib import Path
from typing import Any, List, Literal, Optional

import pydantic
import yaml

from .net_config import MODELS
from .pipeline import DEFAULT_NEGATIVE_PROMPT

IMAGE_EXTENSIONS = [".png", ".jpg", ".jpeg", ".webp"]
VIDEO_EXTENSIONS = [".mp4"]
ModelName = Literal["2B/post-trained", "2B/pre-trained", "14B/pre-trained"]


def is_rank0() -> bool:
    return os.environ.get("RANK", "0") == "0"


def path_to_str(v: Optional[Path]) -> Optional[str]:
    return None if v is None else str(v)


class InferenceType(str, enum.Enum):
    TEXT2WORLD = "text2world"
    IMAGE2WORLD = "image2world"
    VIDEO2WORLD = "video2world"

    def __str__(self) -> str:
        return self.value


INPUT_EXTENSIONS = {
    InferenceType.TEXT2WORLD: None,
    InferenceType.IMAGE2WORLD: IMAGE_EXTENSIONS + VIDEO_EXTENSIONS,
    InferenceType.VIDEO2WORLD: IMAGE_EXTENSIONS + VIDEO_EXTENSIONS,
}


class SetupArguments(pydantic.BaseModel):
    model_config = pydantic.ConfigDict(extra="forbid")

    output_dir: Path
    model: ModelName = "2B/post-trained"
    checkpoint_path: Optional[str] = None
    tokenizer_path: Optional[str] = None
    experiment: Optional[str] = None
    config_file: str = "cosmos_predict2/_src/predict2/configs/video2world/config.py"
    context_parallel_size: Optional[pydantic.PositiveInt] = None
    offload_diffusion_model: bool = False
    offload_tokenizer: bool = False
    offload_text_encoder: bool = False
    disable_guardrails: bool = True  # guardrails are outside this build
    offload_guardrail_models: bool = True
    keep_going: bool = True
    profile: bool = False
    state_t: Optional[int] = None  # latent frames; the reference's experiments use 24 (93 frames)

    @pydantic.model_validator(mode="before")
    @classmethod
    def _defaults(cls, data: Any) -> Any:
        if isinstance(data, dict):
            if data.get("model", "2B/post-trained") not in MODELS:
                raise ValueError(f"unknown model {data.get('model')}")
            if data.get("context_parallel_size") is None:
                data["context_parallel_size"] = int(os.environ.get("WORLD_SIZE", "1"))
            for k in ("checkpoint_path", "tokenizer_path"):
                if data.get(k) is not None and not os.path.exists(data[k]):
                    raise ValueError(f"{k} '{data[k]}' does not exist.")
        return data


class InferenceArguments(pydantic.BaseModel):
    model_config = pydantic.ConfigDict(extra="forbid", frozen=True)

    name: str
    prompt: Optional[str] = None
    prompt_path: Optional[Path] = None
    negative_prompt: str = DEFAULT_NEGATIVE_PROMPT
    seed: int = 0
    guidance: int = pydantic.Field(7, ge=0, le=7)
    inference_type: InferenceType
    input_path: Optional[Path] = None
    resolution: str = "none"
    num_output_frames: pydantic.PositiveInt = 77
    num_steps: pydantic.PositiveInt = 35
    enable_autoregressive: bool = False
    chunk_size: int = 77
    chunk_overlap: int = 1

    @pydantic.model_validator(mode="before")
    @classmethod
    def _prompt(cls, data: Any) -> Any:
        if isinstance(data, dict) and data.get("prompt") is None and data.get("prompt_path") is not None:
            data = dict(data)
            data["prompt"] = Path(data["prompt_path"]).read_text().strip()
        return data

    @pydantic.model_validator(mode="after")
    def _check(self):
        if self.prompt is None:
            raise ValueError("one of prompt / prompt_path is required")
        exts = INPUT_EXTENSIONS[self.inference_type]
        if exts is not None:
            if self.input_path is None:
                raise ValueError(f"input_path is required for inference type {self.inference_type}")
            if self.input_path.suffix not in exts:
                raise ValueError(f"input_path has unsupported file extension '{self.input_path.suffix}'")
        return self

    @cached_property
    def num_input_frames(self) -> int:
        return {InferenceType.TEXT2WORLD: 0, InferenceType.IMAGE2WORLD: 1, InferenceType.VIDEO2WORLD: 2}[
            self.inference_type]

    @classmethod
    def from_files(cls, paths: List[Path], overrides: Optional[dict] = None) -> List["InferenceArguments"]:
        """json / jsonl / yaml sample files (config.py:344-377); input paths relative to the file."""
        out: List[InferenceArguments] = []
        for path in map(Path, paths):
            text = path.read_text()
            if path.suffix == ".json":
                rows = [json.loads(text)]
            elif path.suffix == ".jsonl":
                rows = [json.loads(line) for line in text.splitlines() if line]
            elif path.suffix in (".yaml", ".yml"):
                rows = [yaml.safe_load(text)]
            else:
                raise ValueError(f"Unsupported file extension: {path.suffix}")
            for r in rows:
                r = dict(r, **(overrides or {}))
                for k in ("input_path", "prompt_path"):
                    if r.get(k) is not None and not os.path.isabs(r[k]):
                        r[k] = str((path.parent / r[k]).resolve())
                out.append(cls.model_validate(r))
        names = [o.name for o in out]
        if len(set(names)) != len(names):
            raise ValueError("sample names must be unique")
        return out
