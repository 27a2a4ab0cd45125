"""Video2WorldModelRectifiedFlow for MI355X: conditioning, CFG velocity and the UniPC sampling loop.

Reference: cosmos_predict2/_src/predict2/models/video2world_model_rectified_flow.py (denoise :77-138,
velocity_fn :140-212) and text2world_model_rectified_flow.py (generate_samples_from_batch :516-599,
_normalize_video_databatch_inplace :703-737, encode/decode :864-870).

Hot-loop layout (DESIGN.md "Sampler"): the latent state, the noise and the ground-truth latent live
in HBM in *patch layout* [tokens, 64] fp32 (token = (t, h/2, w/2), feature (p1 p2 C)); a context-
parallel rank owns a contiguous token range. One sampler step is
    patchify (HIP) -> DiT forward on the CFG batch [cond, uncond] (B = 2)
    -> GT-frame velocity replacement + CFG (HIP, reads the final layer's output in place)
    -> fused UniPC corrector/predictor update (HIP)
with the only inter-GPU traffic the K/V all-gather inside self-attention.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from . import _native as N
from . import context_parallel as cpu
from .dit import Geometry, MinimalV1LVGDiT
from .net_config import DiTConfig, SamplerConfig
from .scheduler import FlowUniPCMultistepScheduler

NUM_CONDITIONAL_FRAMES_KEY = "num_conditional_frames"


def arch_invariant_rand(shape, dtype, device, seed: Optional[int] = None) -> torch.Tensor:
    """imaginaire/utils/misc.py:158-179: numpy RandomState noise, identical on every host."""
    rng = np.random.RandomState(seed)
    return torch.from_numpy(rng.standard_normal(shape).astype(np.float32)).to(dtype=dtype, device=device)


def to_patch_layout(x_C_T_H_W: torch.Tensor) -> torch.Tensor:
    """[C=16, T, H, W] -> [T*(H/2)*(W/2), 64] with feature (p1*2 + p2)*16 + c."""
    C, T, H, W = x_C_T_H_W.shape
    return x_C_T_H_W.reshape(C, T, H // 2, 2, W // 2, 2).permute(1, 2, 4, 3, 5, 0).reshape(-1, 4 * C).contiguous()


def from_patch_layout(xp: torch.Tensor, T: int, H: int, W: int) -> torch.Tensor:
    C = xp.shape[1] // 4
    return xp.view(T, H // 2, W // 2, 2, 2, C).permute(5, 0, 1, 3, 2, 4).reshape(C, T, H, W).contiguous()


class Video2WorldModelRectifiedFlow:
    """Inference model: `generate_samples_from_batch`, `denoise`, `encode`, `decode`."""

    def __init__(self, net_cfg: DiTConfig, sampler_cfg: SamplerConfig, tokenizer=None, device="cuda"):
        self.net_cfg = net_cfg
        self.config = sampler_cfg
        self.device = torch.device(device)
        self.net = MinimalV1LVGDiT(net_cfg, device=self.device)
        self.tokenizer = tokenizer
        self.sample_scheduler = FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1)
        self.cp_group = None
        # replay each trajectory's DiT forward from a HIP graph after its first evaluation (SamplingRun; one GPU only):
        # for launch-bound shapes (config 5's 13-frame chunks), where the host's launch rate leaves the device idle
        self.hip_graph = False

    # ------------------------------------------------------------------ plumbing
    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        self.net.load_state_dict(sd, strict=strict)

    def set_context_parallel_group(self, group) -> None:
        self.cp_group = group
        if self.tokenizer is not None and hasattr(self.tokenizer, "set_context_parallel_group"):
            self.tokenizer.set_context_parallel_group(group)
        if group is None:
            self.net.disable_context_parallel()
        else:
            self.net.enable_context_parallel(group)

    @torch.no_grad()
    def encode(self, state: torch.Tensor) -> torch.Tensor:
        return self.tokenizer.encode(state)

    @torch.no_grad()
    def decode(self, latent: torch.Tensor) -> torch.Tensor:
        return self.tokenizer.decode(latent)

    def _normalize_video(self, video: torch.Tensor) -> torch.Tensor:
        # uint8 -> [-1, 1] in bf16 arithmetic (text2world_model_rectified_flow.py:735-736)
        if video.dtype == torch.uint8:
            return video.to(device=self.device, dtype=torch.bfloat16) / 127.5 - 1.0
        return video.to(self.device)

    # ------------------------------------------------------------------ per-frame timesteps
    def _frame_timesteps(self, t: torch.Tensor, frame_mask: torch.Tensor) -> torch.Tensor:
        """denoise :109-122 -> [T] fp32 (cond frames -> conditional_frame_timestep)."""
        tf = t.to(torch.float32).expand(frame_mask.shape[0]).to(frame_mask.device)
        c = self.config.conditional_frame_timestep
        if c >= 0:
            tcond = torch.ones_like(frame_mask) * c
            tf = tcond * frame_mask + t.to(frame_mask.device) * (1 - frame_mask)
        return tf

    # ------------------------------------------------------------------ the sampler
    @torch.no_grad()
    def begin_sampling(self, gt: Optional[torch.Tensor], ctx_cond: torch.Tensor, ctx_uncond: torch.Tensor, *,
                       state_shape, num_conditional_frames: int, guidance: float, seed: int, num_steps: int,
                       shift: float = 5.0, cfg_mode: Optional[str] = None, net_fn=None,
                       action: Optional[torch.Tensor] = None,
                       view_indices: Optional[torch.Tensor] = None) -> "SamplingRun":
        """Set up one trajectory of the sampling loop (text2world_model_rectified_flow.py:556-582):
        noise, schedule, conditioning; SamplingRun.step() then runs one loop iteration (:584-594)."""
        return SamplingRun(self, gt, ctx_cond, ctx_uncond, state_shape=state_shape,
                           num_conditional_frames=num_conditional_frames, guidance=guidance, seed=seed,
                           num_steps=num_steps, shift=shift, cfg_mode=cfg_mode, net_fn=net_fn, action=action,
                           view_indices=view_indices)

    @torch.no_grad()
    def sample_latents(self, gt: Optional[torch.Tensor], ctx_cond: torch.Tensor, ctx_uncond: torch.Tensor, *,
                       state_shape, num_conditional_frames: int, guidance: float, seed: int, num_steps: int,
                       shift: float = 5.0, cfg_mode: Optional[str] = None, progress=None,
                       net_fn=None, action: Optional[torch.Tensor] = None,
                       view_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Core loop. gt: x0 latent [1, C, T, H, W] fp32 (or None when no frame is conditioned);
        ctx_*: text embeddings [1, Lctx, proj_in]. Returns latents [1, C, T, H, W] fp32.
        net_fn(rows [n,1,72] bf16, t_B_T [2,T] fp32, geo) -> [n,2,64] replaces the DiT (tests only)."""
        run = self.begin_sampling(gt, ctx_cond, ctx_uncond, state_shape=state_shape,
                                  num_conditional_frames=num_conditional_frames, guidance=guidance, seed=seed,
                                  num_steps=num_steps, shift=shift, cfg_mode=cfg_mode, net_fn=net_fn,
                                  action=action, view_indices=view_indices)
        while not run.done:
            i = run.step()
            if progress is not None:
                progress(i, run.num_evals)
        return run.latents()

    @torch.no_grad()
    def generate_samples_from_batch(self, data_batch: Dict, guidance: float = 1.5, seed: int = 1,
                                    state_shape=None, n_sample: Optional[int] = None,
                                    is_negative_prompt: bool = False, num_steps: int = 35, shift: float = 5.0,
                                    **kwargs) -> torch.Tensor:
        """text2world_model_rectified_flow.py:516-599 (+ the Video2World velocity_fn)."""
        run = self.begin_sampling_from_batch(data_batch, guidance=guidance, seed=seed, state_shape=state_shape,
                                             is_negative_prompt=is_negative_prompt, num_steps=num_steps, shift=shift)
        while not run.done:
            run.step()
        return run.latents()

    @torch.no_grad()
    def begin_sampling_from_batch(self, data_batch: Dict, guidance: float = 1.5, seed: int = 1, state_shape=None,
                                  is_negative_prompt: bool = False, num_steps: int = 35,
                                  shift: float = 5.0) -> "SamplingRun":
        """generate_samples_from_batch up to its loop: encode the conditioning frames (VAE), build the
        CFG contexts, noise and schedule; returns the steppable SamplingRun."""
        video = data_batch["video"]
        if state_shape is None:
            _T, _H, _W = video.shape[-3:]
            sc = self.tokenizer.spatial_compression_factor
            state_shape = [self.config.state_ch, self.tokenizer.get_latent_num_frames(_T), _H // sc, _W // sc]
        n_cond = data_batch.get(NUM_CONDITIONAL_FRAMES_KEY, 1)
        n_cond = int(n_cond.item()) if isinstance(n_cond, torch.Tensor) else int(n_cond)
        gt = None
        if n_cond > 0:
            gt = self.encode_conditioning(video, n_cond, state_shape[1])
        ctx_c = data_batch["t5_text_embeddings"]
        if is_negative_prompt and isinstance(data_batch.get("neg_t5_text_embeddings"), torch.Tensor):
            ctx_u = data_batch["neg_t5_text_embeddings"]
        else:
            ctx_u = torch.zeros_like(ctx_c)  # TextAttr dropout (rate 0.2 > 0) zeroes the embedding
        # action-conditioned nets: the same action conditions both CFG branches (the conditioner's
        # action ReMapkey has no dropout: action/configs/action_conditioned/conditioner.py:222-233,272-275)
        return self.begin_sampling(gt, ctx_c, ctx_u, state_shape=state_shape, num_conditional_frames=n_cond,
                                   guidance=guidance, seed=seed, num_steps=num_steps, shift=shift,
                                   action=data_batch.get("action"))

    @torch.no_grad()
    def encode_conditioning(self, video: torch.Tensor, n_cond: int, T_lat: int) -> torch.Tensor:
        """x0 latent of the conditioning frames: [1, C, T_lat, H, W] fp32.

        The causal VAE makes latent frame j depend only on pixel frames <= 4j, so encoding the first
        1 + 4 (n_cond - 1) pixel frames yields the reference's first n_cond latent frames bit-for-bit;
        only those frames reach the output (mask-selected in denoise, video2world_model_rectified_flow.py
        :105-107 and :131-136). The remaining latent frames are zero-filled and never read."""
        px = 1 + 4 * (n_cond - 1)
        vid = self._normalize_video(video[:, :, :px])
        lat = self.encode(vid).float()
        B, C, Tc, H, W = lat.shape
        gt = torch.zeros((B, C, T_lat, H, W), dtype=torch.float32, device=self.device)
        gt[:, :, :Tc] = lat
        return gt

    # ------------------------------------------------------------------ reference-compatible pieces
    @torch.no_grad()
    def denoise(self, noise: torch.Tensor, xt_B_C_T_H_W: torch.Tensor, timesteps_B_T: torch.Tensor,
                condition) -> torch.Tensor:
        """Video2WorldModelRectifiedFlow.denoise (:77-138) for one condition (API compatibility;
        the sampler itself runs the fused CFG-batched path). `condition` is a dict with keys
        gt_frames, condition_video_input_mask_B_C_T_H_W, crossattn_emb, padding_mask (optional)."""
        gt = condition["gt_frames"].to(xt_B_C_T_H_W)
        C = xt_B_C_T_H_W.shape[1]
        m = condition["condition_video_input_mask_B_C_T_H_W"].repeat(1, C, 1, 1, 1).type_as(xt_B_C_T_H_W)
        xt = gt * m + xt_B_C_T_H_W * (1 - m)
        if self.config.conditional_frame_timestep >= 0:
            mt = m.mean(dim=[1, 3, 4], keepdim=True)
            tc = torch.ones_like(mt) * self.config.conditional_frame_timestep
            timesteps_B_T = (tc * mt + timesteps_B_T.to(mt.device) * (1 - mt)).squeeze()
            timesteps_B_T = timesteps_B_T.unsqueeze(0) if timesteps_B_T.ndim == 1 else timesteps_B_T
        out = self.net(xt.to(torch.bfloat16), timesteps_B_T, condition["crossattn_emb"],
                       condition_video_input_mask_B_C_T_H_W=condition["condition_video_input_mask_B_C_T_H_W"],
                       padding_mask=condition.get("padding_mask")).float()
        if self.config.denoise_replace_gt_frames:
            out = (noise - gt.type_as(out)) * m + out * (1 - m)
        return out


class SamplingRun:
    """One sampler trajectory of Video2WorldModelRectifiedFlow, advanced one evaluation at a time.

    Setup = text2world_model_rectified_flow.py:556-582 (noise, schedule, conditioning); step() = one
    iteration of the loop at :584-594 (patchify + frame replacement, the CFG-batched DiT forward,
    GT-frame velocity replacement + CFG, fused UniPC update); latents() = :596-599 (CP gather)."""

    def __init__(self, model: "Video2WorldModelRectifiedFlow", gt, ctx_cond, ctx_uncond, *, state_shape,
                 num_conditional_frames: int, guidance: float, seed: int, num_steps: int, shift: float = 5.0,
                 cfg_mode: Optional[str] = None, net_fn=None, action=None, view_indices=None):
        self.model = model
        C, T, H, W = state_shape
        self.state_shape = (C, T, H, W)
        dev = model.device
        geo = Geometry(T=T, Hp=H // 2, Wp=W // 2, n_views=model.net.n_views_for(T))
        L = geo.L
        cp = model.cp_group
        rank, world = (0, 1) if cp is None else (torch.distributed.get_rank(cp), torch.distributed.get_world_size(cp))
        if L % world:
            raise ValueError(f"token count {L} not divisible by the context-parallel size {world}")
        if world > 1 and model.net.cfg.cross_view_attn_map:
            # cross-view nets shard by frame: every view's frames [rank Tl, (rank + 1) Tl) (Geometry.frame_shard)
            geo = Geometry.frame_shard(T, H // 2, W // 2, geo.n_views, rank, world)
            sl = geo.token_ids(dev)
        else:
            geo.n_tok = L // world
            geo.tok0 = rank * geo.n_tok
            sl = slice(geo.tok0, geo.tok0 + geo.n_tok)
        self.geo, self.cp, self.world = geo, cp, world

        noise_full = arch_invariant_rand((1, C, T, H, W), torch.float32, dev, seed)
        self.noise = to_patch_layout(noise_full[0])[sl].contiguous()
        del noise_full
        frame_mask = torch.zeros(T, dtype=torch.float32, device=dev)
        if geo.T_view > 1 and num_conditional_frames > 0:
            # the first frames of every view (multi-view FIRST_RANDOM_N, predict2_multiview/configs/vid2vid/
            # defaults/conditioner.py:125-260; one view: video2world conditioner.py:45-143)
            for vi in range(geo.n_views):
                frame_mask[vi * geo.T_view: vi * geo.T_view + num_conditional_frames] = 1.0
        self.frame_mask = frame_mask
        # the per-token kernels (patchify, cfg_velocity) index the mask by (tok0 + token) // hw: a frame-sharded rank
        # passes its own frames' entries with tok0 = 0
        self.kmask = frame_mask if geo.frames is None else frame_mask[list(geo.frames)].contiguous()
        self.gtp = None
        if gt is not None and num_conditional_frames > 0:
            self.gtp = to_patch_layout(gt[0].to(dev, torch.float32))[sl].contiguous()

        self.net_fn = net_fn
        self.ctx = None if net_fn is not None else model.net.prepare_context(torch.cat([ctx_cond, ctx_uncond], 0))
        self.mode = 0 if (cfg_mode or model.config.cfg_mode) == "video2world" else 1
        self.guidance = guidance
        # on the device once (a per-evaluation host copy would also be a pageable copy inside a HIP graph capture)
        self.action = None if action is None else action.to(dev)
        self.view_indices = view_indices
        self._sched_args = dict(num_inference_steps=num_steps, device=dev, shift=shift,
                                use_kerras_sigma=model.config.use_kerras_sigma_at_inference)
        # the run's own solver (configured like the model's sample_scheduler): its UniPC history must not be shared
        # with another live run, nor with a sample_latents call made while this run is alive
        base = model.sample_scheduler
        self.sched = FlowUniPCMultistepScheduler(base.num_train_timesteps, base.solver_order, base.config_shift)
        # HIP graph of the DiT forward (model.hip_graph): captured at the second evaluation, after the first one ran
        # eagerly and built every lazily made buffer (RoPE tables, bf16 weight copies), then replayed on static copies
        # of the two inputs that change per evaluation (patch rows, timesteps); the context, the action and every
        # weight stay the tensors the graph recorded. Not with CP (the K/V gathers run on their own streams).
        self._graphable = bool(getattr(model, "hip_graph", False)) and net_fn is None and world == 1
        self._graph = None
        self.restart()

    def restart(self) -> None:
        """Back to the first timestep from the same noise (bench: more evaluations than one trajectory)."""
        sched = self.sched
        sched.set_timesteps(**self._sched_args)
        self.timesteps = sched.timesteps.cpu()
        self.x = sched.begin(self.noise)
        self.i = 0

    @property
    def num_evals(self) -> int:
        return len(self.timesteps)

    @property
    def done(self) -> bool:
        return self.i >= len(self.timesteps)

    @torch.no_grad()
    def step(self) -> int:
        """One sampler evaluation; returns its index in the schedule."""
        if self.done:
            raise RuntimeError("the trajectory is complete (restart() to run it again)")
        m, geo = self.model, self.geo
        t = self.timesteps[self.i]
        rows = N.patchify(self.x, self.gtp, self.kmask, None, tok0=geo.tok0, hw=geo.hw, ld=128)
        tf = m._frame_timesteps(t, self.frame_mask)  # [T]
        t_B_T = m.net.scale_timesteps(tf[None, :]).expand(2, geo.T).contiguous()
        if self.net_fn is None:
            # one t row expanded over the CFG pair, one action: the entries differ only in the text context
            shared = self.action is None or self.action.shape[0] == 1

            def forward(rows_, t_):
                return m.net.forward_tokens(rows_, t_, self.ctx, geo, action=self.action,
                                            view_indices=self.view_indices, shared_batch=shared, rows_k128=True)
            if self._graphable and self.i >= 1:
                # rows is the [n, 72] view of patchify's zero-padded [n, 128] buffer (rows_k128): the static copy
                # keeps that layout, pad columns included
                padded = torch.as_strided(rows, (rows.shape[0], rows.stride(0)), (rows.stride(0), 1))
                if self._graph is None:
                    self._g_buf, self._g_t = padded.clone(), t_B_T.clone()
                    self._g_rows = self._g_buf[:, :rows.shape[1]].view(geo.n_tok, 1, -1)
                    self._graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self._graph):
                        self._g_out = forward(self._g_rows, self._g_t)
                self._g_buf.copy_(padded)
                self._g_t.copy_(t_B_T)
                self._graph.replay()
                net_out = self._g_out
            else:
                net_out = forward(rows.view(geo.n_tok, 1, -1), t_B_T)
        else:
            net_out = self.net_fn(rows.view(geo.n_tok, 1, -1), t_B_T, geo)
        v = N.cfg_velocity(net_out, self.noise, self.gtp, self.kmask, self.guidance, self.mode,
                           tok0=geo.tok0, hw=geo.hw)
        del net_out
        self.sched.step_(v, t)
        self.i += 1
        return self.i - 1

    @torch.no_grad()
    def latents(self) -> torch.Tensor:
        """The current latent state [1, C, T, H, W] fp32 (all-gathered over the CP group)."""
        x = self.x
        if self.world > 1:
            x = cpu.gather_tokens(x, self.cp)
            if self.geo.frames is not None:  # frame-sharded ranks: back to the global (view, frame, h, w) order
                C_, T_, H_, W_ = self.state_shape
                g = self.geo
                ids = torch.cat([Geometry.frame_shard(T_, g.Hp, g.Wp, g.n_views, r, self.world).token_ids(x.device)
                                 for r in range(self.world)])
                xg = torch.empty_like(x)
                xg[ids] = x
                x = xg
        _, T, H, W = self.state_shape
        return from_patch_layout(x, T, H, W).unsqueeze(0)
