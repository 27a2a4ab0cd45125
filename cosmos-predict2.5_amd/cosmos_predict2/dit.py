"""MiniTrainDIT / MinimalV1LVGDiT denoiser for MI355X.

Same checkpoint layout and forward semantics as the reference network
(cosmos_predict2/_src/predict2/networks/minimal_v4_dit.py:1250-1663 and minimal_v1_lvg_dit.py:22-62),
re-designed for the sampler hot path:

* token-major activations [tokens, B, D] (CFG cond/uncond as batch B = 2, batch inner), so a
  context-parallel shard is a contiguous token range and every GEMM is one [tokens*B, K] x [K, N];
* every block op is HIP (libcp25.so): the six projections on a hand-written MFMA GEMM with fused epilogues
  (exact GELU on MLP layer1; the gated residual on the output / cross-output / layer2 projections), LayerNorm +
  AdaLN modulate, per-head RMSNorm + 3D RoPE writing bf16 q/k in place in the fused QKV buffer, flash attention
  reading q/k/v straight out of that buffer; the embedders, AdaLN-LoRA and final linear stay on hipBLASLt;
* everything that is constant across the 36 sampler steps is computed once: the crossattn_proj
  text projection, the cross-attention K/V of every block (per prompt), the RoPE cos/sin tables;
* AdaLN modulation of all blocks in two batched fp32 GEMMs per forward (reference: fp32 autocast).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from . import _native as N
from .context_parallel import all_gather_into_async, kv_chunk_views, run_lanes
from .net_config import DiTConfig

BF16 = torch.bfloat16
F32 = torch.float32


# ----------------------------------------------------------------------------- weights
def state_dict_shapes(cfg: DiTConfig) -> Dict[str, Tuple[Tuple[int, ...], torch.dtype]]:
    """The reference's `net.*` state-dict layout (module names at minimal_v4_dit.py)."""
    D, A, Ctx = cfg.model_channels, cfg.adaln_lora_dim, cfg.crossattn_emb_channels
    hd = cfg.head_dim
    dim_h = hd // 6 * 2
    dim_t = hd - 2 * dim_h
    len_max = max(cfg.max_img_h // cfg.patch_spatial, cfg.max_img_w // cfg.patch_spatial,
                  cfg.max_frames // cfg.patch_temporal)
    s: Dict[str, Tuple[Tuple[int, ...], torch.dtype]] = {
        "x_embedder.proj.1.weight": ((D, cfg.patch_features), BF16),
        "pos_embedder.seq": ((len_max,), BF16),
        "pos_embedder.dim_spatial_range": ((dim_h // 2,), BF16),
        "pos_embedder.dim_temporal_range": ((dim_t // 2,), BF16),
        "t_embedder.1.linear_1.weight": ((D, D), BF16),
        "t_embedder.1.linear_2.weight": ((3 * D, D), BF16),
        "t_embedding_norm.weight": ((D,), BF16),
        "final_layer.linear.weight": ((cfg.patch_spatial ** 2 * cfg.patch_temporal * cfg.out_channels, D), BF16),
        "final_layer.adaln_modulation.1.weight": ((A, D), BF16),
        "final_layer.adaln_modulation.2.weight": ((2 * D, A), BF16),
    }
    if cfg.use_crossattn_projection:
        s["crossattn_proj.0.weight"] = ((Ctx, cfg.crossattn_proj_in_channels), BF16)
        s["crossattn_proj.0.bias"] = ((Ctx,), BF16)
    for i in range(cfg.num_blocks):
        p = f"blocks.{i}."
        for a in ("self_attn", "cross_attn"):
            kv_in = D if a == "self_attn" else Ctx
            s[p + a + ".q_proj.weight"] = ((D, D), BF16)
            s[p + a + ".k_proj.weight"] = ((D, kv_in), BF16)
            s[p + a + ".v_proj.weight"] = ((D, kv_in), BF16)
            s[p + a + ".output_proj.weight"] = ((D, D), BF16)
            s[p + a + ".q_norm.weight"] = ((hd,), BF16)
            s[p + a + ".k_norm.weight"] = ((hd,), BF16)
        if cfg.cross_view_attn_map:  # MultiViewCrossBlock (multiview_cross_dit.py:282-290)
            for m in ("q_proj", "k_proj", "v_proj", "output_proj"):
                s[p + f"cross_view_attn.{m}.weight"] = ((D, D), BF16)
            s[p + "cross_view_attn.q_norm.weight"] = ((hd,), BF16)
            s[p + "cross_view_attn.k_norm.weight"] = ((hd,), BF16)
            s[p + "layer_norm_cross_view_attn.weight"] = ((D,), BF16)
            s[p + "layer_norm_cross_view_attn.bias"] = ((D,), BF16)
        s[p + "mlp.layer1.weight"] = ((cfg.mlp_hidden, D), BF16)
        s[p + "mlp.layer2.weight"] = ((D, cfg.mlp_hidden), BF16)
        for m in ("self_attn", "cross_attn", "mlp"):
            s[p + f"adaln_modulation_{m}.1.weight"] = ((A, D), BF16)
            s[p + f"adaln_modulation_{m}.2.weight"] = ((3 * D, A), BF16)
    if cfg.n_cameras_emb and cfg.view_condition_dim:
        s["view_embeddings.weight"] = ((cfg.n_cameras_emb, cfg.view_condition_dim), BF16)
    if cfg.adaln_view_embedding:  # multiview_cross_dit.py:575-579
        s["adaln_view_embedder.weight"] = ((cfg.n_cameras_emb, D), BF16)
        s["adaln_view_proj.weight"] = ((9 * D, D), BF16)
        s["adaln_view_proj.bias"] = ((9 * D,), BF16)
    if cfg.action_dim:
        fin, hid = cfg.action_in_features, cfg.action_hidden_features
        for name, out in (("action_embedder_B_D", D), ("action_embedder_B_3D", 3 * D)):
            s[name + ".fc1.weight"] = ((hid, fin), BF16)
            s[name + ".fc1.bias"] = ((hid,), BF16)
            s[name + ".fc2.weight"] = ((out, hid), BF16)
            s[name + ".fc2.bias"] = ((out,), BF16)
    return s


def init_state_dict(cfg: DiTConfig, seed: int = 0, device="cpu", zero_adaln_out: bool = True) -> Dict[str, torch.Tensor]:
    """Seeded synthetic weights with the reference's init_weights distributions
    (minimal_v4_dit.py:239-247, 386-398, 769-774, 887-889, 954-963, 1100-1122, 1445-1459).
    zero_adaln_out=False fills the zero-initialised AdaLN output layers too (exercises the path)."""
    g = torch.Generator(device=device).manual_seed(seed)
    out: Dict[str, torch.Tensor] = {}

    def tn(shape, std):
        t = torch.empty(shape, dtype=F32, device=device)
        torch.nn.init.trunc_normal_(t, std=std, a=-3 * std, b=3 * std, generator=g)
        return t.to(BF16)

    D = cfg.model_channels
    shapes = state_dict_shapes(cfg)
    shapes_fan = {k: shapes[k[: k.rindex(".")] + ".weight"][0][1] for k in shapes if k.startswith("action_embedder")}
    for name, (shape, _) in shapes.items():
        if name.endswith("norm.weight"):
            out[name] = torch.ones(shape, dtype=BF16, device=device)
        elif name == "pos_embedder.seq":
            out[name] = torch.arange(shape[0], device=device).float().to(BF16)
        elif name.startswith("pos_embedder.dim_"):
            full = 2 * shape[0] if "spatial" in name else 2 * shape[0]
            out[name] = (torch.arange(0, full, 2, device=device)[: shape[0]].float() / full).to(BF16)
        elif name == "view_embeddings.weight":  # multiview_dit.py:390-391
            out[name] = (torch.randn(shape, generator=g, device=device) * 0.02).to(BF16)
        elif name == "adaln_view_embedder.weight":  # multiview_cross_dit.py:664-665
            out[name] = (torch.randn(shape, generator=g, device=device) * 0.05).to(BF16)
        elif name.startswith("adaln_view_proj") or name.endswith("cross_view_attn.output_proj.weight"):
            # zero-initialised (:667-669, :306-309); zero_adaln_out=False fills them to exercise the path
            out[name] = (torch.zeros(shape, dtype=BF16, device=device) if zero_adaln_out else
                         tn(shape, 0.02 if name.endswith("bias") else 1.0 / math.sqrt(D)))
        elif "layer_norm_cross_view_attn" in name:  # nn.LayerNorm init (1, 0); perturbed with zero_adaln_out=False
            base = 1.0 if name.endswith("weight") else 0.0
            noise = 0.0 if zero_adaln_out else 0.1
            out[name] = (base + noise * torch.randn(shape, generator=g, device=device)).to(BF16)
        elif name.startswith("action_embedder"):  # nn.Linear default init (not covered by init_weights)
            fan_in = shapes_fan[name]
            bound = 1.0 / math.sqrt(fan_in)
            out[name] = (torch.rand(shape, generator=g, device=device) * 2 - 1).mul_(bound).to(BF16)
        elif name.startswith("crossattn_proj"):
            bound = 1.0 / math.sqrt(cfg.crossattn_proj_in_channels)
            out[name] = (torch.rand(shape, generator=g, device=device) * 2 - 1).mul_(bound).to(BF16)
        elif name.endswith(".2.weight") and "adaln_modulation" in name and zero_adaln_out:
            out[name] = torch.zeros(shape, dtype=BF16, device=device)
        else:
            fan_in = shape[1]
            out[name] = tn(shape, 1.0 / math.sqrt(fan_in if "output_proj" not in name else D))
    return out


# ----------------------------------------------------------------------------- RoPE
def rope_freqs(cfg: DiTConfig, T: int, H: int, W: int, sd: Dict[str, torch.Tensor], device) -> torch.Tensor:
    """VideoRopePosition3DEmb.generate_embeddings (minimal_v4_dit.py:598-663) with the bf16 range
    buffers of the checkpoint (F8): -> [T*H*W, head_dim] fp32."""
    hd = cfg.head_dim
    dim_h = hd // 6 * 2
    dim_t = hd - 2 * dim_h
    seq = sd["pos_embedder.seq"].to(device)
    rs = sd["pos_embedder.dim_spatial_range"].to(device).float()
    rt = sd["pos_embedder.dim_temporal_range"].to(device).float()
    h_theta = 10000.0 * cfg.rope_h_extrapolation_ratio ** (dim_h / (dim_h - 2))
    w_theta = 10000.0 * cfg.rope_w_extrapolation_ratio ** (dim_h / (dim_h - 2))
    t_theta = 10000.0 * cfg.rope_t_extrapolation_ratio ** (dim_t / (dim_t - 2))
    if H > cfg.max_img_h // cfg.patch_spatial or W > cfg.max_img_w // cfg.patch_spatial:
        raise ValueError(f"latent patches ({H}, {W}) exceed the RoPE table")
    eh = torch.outer(seq[:H], 1.0 / (h_theta ** rs))
    ew = torch.outer(seq[:W], 1.0 / (w_theta ** rs))
    et = torch.outer(seq[:T], 1.0 / (t_theta ** rt))
    em = torch.cat([et[:, None, None].expand(T, H, W, -1), eh[None, :, None].expand(T, H, W, -1),
                    ew[None, None, :].expand(T, H, W, -1)] * 2, dim=-1)
    return em.reshape(T * H * W, hd).float()


@dataclass
class ContextCache:
    """Per-prompt constants: projected text context and every block's cross-attention K/V."""

    B: int
    k: List[torch.Tensor]  # [B, Lctx, H, hd] bf16 (normed)
    v: List[torch.Tensor]  # [B, Lctx, H, hd] bf16


@dataclass
class Geometry:
    T: int   # latent frames (patches along t)
    Hp: int  # patches along h
    Wp: int  # patches along w
    tok0: int = 0  # first global token of this rank's shard
    n_tok: int = 0  # tokens on this rank
    n_views: int = 1  # multi-view: T = n_views x per-view frames, tokens ordered (view, t, h, w)
    # frame-sharded rank (cross-view nets under context parallelism, frame_shard): the global frame of each local frame,
    # local tokens ordered (view, local frame, h, w); None = the contiguous token range [tok0, tok0 + n_tok)
    frames: Optional[Tuple[int, ...]] = None

    @classmethod
    def frame_shard(cls, T: int, Hp: int, Wp: int, n_views: int, rank: int, world: int) -> "Geometry":
        """Rank `rank` of `world` holds frames [rank Tl, (rank + 1) Tl) of every view (Tl = T / n_views / world): the
        reference's multi-view CP layout ("B C (c V T) H W", multiview_vid2vid_model_rectified_flow.py:400-403), in
        which the cross-view attention of a frame needs no other rank (CrossViewAttention.set_context_parallel_group,
        multiview_cross_dit.py:230-231) and each view's self-attention gathers the other ranks' frames."""
        Tv = T // n_views
        if T % n_views or Tv % world:
            raise ValueError(f"{T} frames of {n_views} views do not shard by frame over {world} ranks")
        Tl = Tv // world
        frames = tuple(v * Tv + rank * Tl + t for v in range(n_views) for t in range(Tl))
        return cls(T=T, Hp=Hp, Wp=Wp, tok0=0, n_tok=len(frames) * Hp * Wp, n_views=n_views, frames=frames)

    def token_ids(self, device=None) -> torch.Tensor:
        """Global token index of each local token."""
        if self.frames is None:
            return torch.arange(self.tok0, self.tok0 + self.n_tok, device=device)
        f = torch.tensor(self.frames, device=device)
        return (f[:, None] * self.hw + torch.arange(self.hw, device=device)[None, :]).reshape(-1)

    def local(self) -> "Geometry":
        """A frame-sharded rank's tokens as a geometry of their own (T = its frames, tok0 = 0); else self."""
        if self.frames is None:
            return self
        return Geometry(T=len(self.frames), Hp=self.Hp, Wp=self.Wp, tok0=0, n_tok=self.n_tok, n_views=self.n_views)

    @property
    def T_view(self) -> int:
        return self.T // self.n_views

    @property
    def L_view(self) -> int:
        return self.L // self.n_views

    @property
    def hw(self) -> int:
        return self.Hp * self.Wp

    @property
    def L(self) -> int:
        return self.T * self.Hp * self.Wp


def _require_gemm(w: torch.Tensor, what: str = "projection") -> None:
    """Every linear of the sampler runs on a hand-written GEMM, with no library fallback: a weight [N, K] whose shape
    cp25_gemm_epi is not built for (N a multiple of 256, K of 64) raises ValueError, as a missing libcp25.so does."""
    n_out, k = w.shape
    if not N.gemm_supported(n_out, k):
        raise ValueError(f"{what} weight [{n_out}, {k}]: the own GEMM needs N % 256 == 0 and K % 64 == 0")


def _rows(h, m: int):
    """[m, D] rows of an LN-mod output: a bf16 [n, B, D] tensor, or an fp8 (q, scale) pair as is."""
    return h if isinstance(h, tuple) else h.view(m, -1)


class MinimalV1LVGDiT:
    """Inference-only DiT with the reference's state-dict layout; weights live in HBM as bf16."""

    def __init__(self, cfg: DiTConfig, device="cuda"):
        if cfg.head_dim != 128:
            raise ValueError("the MI355X attention kernel is built for head_dim 128 (2B and 14B both use it)")
        if cfg.patch_temporal != 1 or cfg.patch_spatial != 2 or cfg.out_channels != 16:
            raise ValueError("patch (1,2,2) with 16 latent channels is the layout this build serves")
        self.cfg = cfg
        self.device = torch.device(device)
        self.sd: Dict[str, torch.Tensor] = {}
        self._rope_cache: Dict[Tuple[int, int, int], Tuple[torch.Tensor, torch.Tensor]] = {}
        self.cp_group = None
        self.force_lanes = False  # run the per-batch-entry lanes at CP = 1 too (CP parity tests)
        # optional list collecting (start, end, flop) HIP events around every self-attention launch
        self.attn_events: Optional[list] = None
        # optional list collecting (start, end) HIP events around every context-parallel K/V gather wait on the compute
        # stream: the time the stream stood still for the all-gather, i.e. the communication the lanes did not hide
        self.comm_events: Optional[list] = None
        # "bf16" (the reference's precision) or "fp8": the block projections and MLP as fp8 MFMA GEMMs
        # with row-scaled activations and per-output-channel weight scales (config 5, see set_linear_precision)
        self.linear_precision = "bf16"
        self._fp8_w: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
        # True: self-attention q rounded to bf16 exactly where the reference rounds it (the scale goes
        # on the fp32 scores); False (default): q * scale * log2(e) rounded once (see _self_attn_mode)
        self.exact_q_rounding = False
        # "bf16" (default), "fp8qk" (self-attention Q K^T on e4m3) or "fp8" (also P.V on e5m2 P, e4m3 V)
        self.attention_precision = "bf16"
        # the CFG pair's shared block-0 prefix runs once (see _blocks); False: every entry computes it
        self.share_cfg_block0 = True
        # single-GPU self-attention with weight-based norm bounds past the zero-shift window (trained q/k norm weights):
        # True (default since round 6): the k RMSNorm kernel measures max |k| (64 device slots) and the attention runs
        # the gated pair, the fixed-shift loop on that measured bound for every 256-query block it allows (<= 110 in
        # log2 units; small P, no running max), the online max for the rest (cp25_attn_fwd_prescaled_kslots): -0.83 %
        # per sampler evaluation against the online max with norm weights in [0.5, 3], the k norm's separate max-|k|
        # pass included (profiles/r6/shift_power/ab_in_dit_trained.json). False: the online max, whose rows never
        # depend on their 256-row block or on the other CFG entry's keys. Context-parallel shards always take the
        # weight bounds (the CP path does not read this flag), so they stay bit-identical to a CP = 1 run with it off
        # (tests/test_cp_gpu.py "nw_weight") -- under CP25_ATTN_SPLIT=1 only: by default the attention's tail split
        # (cp25_attn_tail_workspace_bytes) runs the query blocks of a launch's last partial round as key-range splits,
        # and which blocks those are depends on the launch's workgroup count mod the CU count, so it differs between
        # CP = 1 and a shard (and between GPUs with different CU counts); those rows then differ from the unsplit ones by
        # rounding (the same distance from fp32, tests/test_attn_m16_gpu.py)
        self.data_tight_k_bound = True
        # the self-attention normalises its own q (cp25_attn_fwd_prescaled_qnorm: head_rmsnorm_rope's arithmetic on
        # the Q fragments as they load, bit-identical, no separate pass over q in HBM); prescaled bf16 form only
        self.fused_q_norm = True
        self._x_embed_w128 = None  # the x_embedder weight zero-padded to K = 128 (embed_patches' own-GEMM path)

    def set_linear_precision(self, precision: str) -> None:
        """"bf16" (default, the reference's arithmetic) or "fp8": the 28 blocks' q/k/v, output, cross-q,
        cross-output and MLP projections run as fp8 (OCP E4M3) MFMA GEMMs, the hand-written cp25_gemm_fp8 (with the
        gated residual fused into the output projections' epilogue, cp25_gemm_fp8_res; a ValueError for shapes it is
        not built for), activations quantised per row by cp25_quant_fp8_rows (the MLP's
        fused with its GELU, cp25_gelu_quant_fp8), weights per output channel (once, on first use). Embedders, AdaLN, the text projection and the final layer
        stay bf16/fp32. The reference has no fp8 path: the cost is stated against the bf16 path
        (DESIGN.md §4), not pinned to a reference output."""
        if precision not in ("bf16", "fp8"):
            raise ValueError(f"linear precision must be 'bf16' or 'fp8', got {precision!r}")
        self.linear_precision = precision
        self._fp8_w = {}

    def set_attention_precision(self, precision: str) -> None:
        """"bf16" (default, the reference's arithmetic), "fp8qk" or "fp8" (config 5's option; no reference
        counterpart). Where the prescaled form applies, "fp8qk" runs the self-attention's Q K^T on
        v_mfma_f32_32x32x64_f8f6f4 over e4m3 copies of q * 4 and k / 4 (cp25_cast_fp8_e4m3, power-of-two scales
        that cancel in the scores; cp25_attn_fwd_prescaled_fp8qk), P and V bf16: -18 % on the kernel. "fp8"
        also runs P.V in fp8 (cp25_attn_fwd_prescaled_fp8: P = exp2(S - shift) as e5m2, V as e4m3 with a
        per-head scale, cp25_cast_v_fp8t): -38 %. The softmax stays fp32. The cost at full depth is stated in
        tests/test_parity_depth_gpu.py::test_full_depth_2b_forward_fp8_modes."""
        if precision not in ("bf16", "fp8qk", "fp8"):
            raise ValueError(f"attention precision must be 'bf16', 'fp8qk' or 'fp8', got {precision!r}")
        self.attention_precision = precision

    def _fp8_qk(self, q_cols: torch.Tensor, k_cols: torch.Tensor, B: int, H: int, hd: int, attn_kw: dict,
                v: Optional[torch.Tensor] = None):
        """attn_fwd kwargs of the prescaled self-attention beyond the bf16 views: the fp8 forms' e4m3 [n, B, H, hd]
        copies of the q / k columns (2-D row views of the token-major qkv / gathered kv buffers), transposed like the
        bf16 views, and for "fp8" also the e4m3 V^T tiles of v. Each fp8 form runs only where its fixed softmax
        window holds every row (the library's rule: bound product <= 60 for fp8 Q K^T, 1.13 x it <= 30 for fp8 P.V,
        whose e5m2 P spans 2^-15 .. 2^15); beyond that the next wider form runs (fp8 -> fp8qk -> bf16)."""
        if not attn_kw.get("prescaled") or self.attention_precision == "bf16":
            return attn_kw
        qb, kb = attn_kw["norm_bounds"]
        if qb * kb > 60.0:
            return attn_kw
        q8 = N.cast_fp8(q_cols, 4.0).view(-1, B, H, hd).transpose(0, 1)
        k8 = N.cast_fp8(k_cols, 0.25).view(-1, B, H, hd).transpose(0, 1)
        kw = dict(attn_kw, fp8_qk=(q8, k8))
        if self.attention_precision == "fp8" and 1.13 * qb * kb <= 30.0:
            kw["fp8_v"] = N.cast_v_fp8t(v)
        return kw

    def _q_norm_in_attention(self, attn_kw: dict) -> bool:
        """The self-attention launch applies the q RMSNorm + RoPE itself (fused_q_norm, prescaled bf16 form)."""
        return self.fused_q_norm and attn_kw.get("prescaled", False) and self.attention_precision == "bf16"

    def _self_attn_mode(self, i: int, hd: int):
        """(q out_scale, attn_fwd kwargs) of block i's self-attention. q leaves the RMSNorm/RoPE kernel as
        bf16(q * hd^-0.5 * log2(e)) and the attention runs without a per-score multiply (cp25_attn_fwd_prescaled):
        the softmax shift rides in the Q K^T chains' initial C, fixed from the weight norm bounds where they allow
        it (bound product <= 96 in log2 units: norm weights up to ~2.4, e.g. the unit init weights) and an online row max otherwise (trained
        q/k norm weights of any size). Rounding q * c instead of q to bf16 is the same single bf16 rounding of the
        query at the same relative size, so the distance to the fp32 truth is unchanged
        (tests/test_parity_depth_gpu.py holds the HIP path within 1.1x of the bf16 reference's own distance);
        `exact_q_rounding = True` keeps the reference's rounding point (q rounded, scale applied to the fp32
        scores)."""
        return self._attn_mode(self.attn_bounds[i], hd)

    def _k_slots(self, attn_kw: dict) -> Optional[torch.Tensor]:
        """Zeroed max-|k| slots for a prescaled bf16 self-attention whose weight-based bounds exceed the zero-shift
        window (data_tight_k_bound), else None. Single-GPU only: the gated pair picks a row's mode per 256-query
        block, which context-parallel shards (bit-identical to CP = 1 by contract) must not depend on."""
        if not (self.data_tight_k_bound and attn_kw.get("prescaled") and self.attention_precision == "bf16"):
            return None
        qb, kb = attn_kw["norm_bounds"]
        if qb * kb <= 110.0:  # the weight bounds already give the fixed shift (attn_fwd.hip m16_mode, kGateFixed)
            return None
        return torch.zeros((64, 32), dtype=torch.float32, device=self.device)

    def _attn_mode(self, bounds, hd: int):
        """The rule of _self_attn_mode for any RMS-normed q / k pair (also the text cross-attention)."""
        qb, kb = bounds
        c = hd ** -0.5 * 1.4426950408889634
        if not self.exact_q_rounding:
            return c, dict(norm_bounds=(qb * c, kb), prescaled=True)
        return 1.0, dict(softmax_scale=hd ** -0.5, norm_bounds=(qb, kb))

    def _fp8_weight(self, key: str, w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        ent = self._fp8_w.get(key)
        if ent is None:
            fmax = torch.finfo(torch.float8_e4m3fn).max
            wf = w.float()
            sc = (wf.abs().amax(dim=1, keepdim=True) / fmax).clamp_min(torch.finfo(torch.float32).tiny)
            w8 = (wf / sc).clamp(-fmax, fmax).to(torch.float8_e4m3fn)
            ent = (w8, sc.t().contiguous())  # [N, K] fp8, [1, N] fp32
            self._fp8_w[key] = ent
        return ent

    def _own(self, x, w: torch.Tensor) -> bool:
        """True: a bf16 projection, on the hand-written bf16 GEMM (cp25_gemm_*); False: the fp8 option's operands.
        Every projection runs on a hand-written GEMM: a weight shape it is not built for raises ValueError."""
        if isinstance(x, tuple) or self.linear_precision != "bf16":
            return False
        _require_gemm(w)
        return True

    def _own_fp8(self, w: torch.Tensor) -> bool:
        """True under the fp8 option (the hand-written cp25_gemm_fp8; ValueError for a shape it is not built for)."""
        if self.linear_precision != "fp8":
            return False
        if not N.gemm_fp8_supported(w.shape[0], w.shape[1]):
            raise ValueError(f"fp8 projection weight {tuple(w.shape)}: cp25_gemm_fp8 needs N and K multiples of 256")
        return True

    def _fused_res(self, a, w: torch.Tensor, B: int, hw: int) -> int:
        """Which hand-written GEMM carries this projection's gated residual in its epilogue: 1 bf16 (cp25_gemm_res),
        2 fp8 (cp25_gemm_fp8_res), 0 none (the plain GEMM, the residual in cp25_ln_mod / the final layer). Both need
        16 % B == 0 and at least 16 / B tokens per frame (N.gemm_res_supported)."""
        if not N.gemm_res_supported(w.shape[0], w.shape[1], B, hw):
            return 0
        return 1 if self._own(a, w) else (2 if self._own_fp8(w) else 0)

    def _proj(self, x, w: torch.Tensor, key: str) -> torch.Tensor:
        """A block projection without epilogue (QKV, cross-attention q)."""
        return N.gemm_epi(x, w) if self._own(x, w) else self._linear(x, w, key)

    def _qkv_k_normed(self, h, i: int, n_rows: int, B: int, cos, sin, kslots=None) -> torch.Tensor:
        """Block i's fused q|k|v projection [n_rows, 3D] with k RMSNorm'd + RoPE'd: in the own GEMM's epilogue
        (cp25_gemm_qkv, bit-identical) where it applies, else the projection and the k pass of cp25_head_rmsnorm_rope
        (which also fills the data-tight key-bound slots when kslots is given)."""
        cfg = self.cfg
        D, H = cfg.model_channels, cfg.num_heads
        x, w, kw = _rows(h, n_rows), self.w_qkv[i], self.sd[f"blocks.{i}.self_attn.k_norm.weight"]
        if kslots is None and self._own(x, w):
            qkv = N.gemm_qkv(x, w, kw, k_col0=D, k_cols=D, B=B, cos=cos, sin=sin)
            if qkv is not None:
                return qkv
        qkv = self._proj(x, w, f"qkv.{i}")
        N.head_rmsnorm_rope(qkv, n_rows=n_rows, B=B, H=H, head_off=D, weight=kw, cos=cos, sin=sin,
                            **({} if kslots is None else dict(norm_max=kslots)))
        return qkv

    def _proj_res(self, a, w: torch.Tensor, key: str, x: torch.Tensor, x_st: int, x_sb: int, gate: torch.Tensor,
                  B: int, geo: "Geometry", n: int, lnk: dict, shift=None, scale=None, gelu_in: bool = False):
        """x' = x + gate * (a w^T) (Block.forward's gated residuals, minimal_v4_dit.py:1204, 1237, 1246) for the token-
        major [n, B, D] rows, then (if shift is given) h = LN-mod(x') for the next sub-layer. Own GEMM: the residual
        rides in its epilogue (cp25_gemm_res) and the LN-mod reads x' only; else the plain own GEMM + the residual
        in cp25_ln_mod. Returns (x' [n, B, D], h or None)."""
        D = w.shape[0]
        fused = None
        path = self._fused_res(a, w, B, geo.hw)
        if path == 1:
            fused = N.gemm_res(a, w, x, x_st, x_sb, gate, B=B, tok0=geo.tok0, hw=geo.hw)
        elif path == 2:
            q, s = a if isinstance(a, tuple) else N.quant_fp8_rows(a, gelu=gelu_in)
            w8, ws = self._fp8_weight(key, w)
            fused = N.gemm_fp8(q, s, w8, ws, res=(x, x_st, x_sb, gate, B, geo.tok0, geo.hw))
        if fused is not None:
            x_new = fused.view(n, B, D)
            h = None
            if shift is not None:
                h = N.ln_mod(x_new, shift, scale, x_st=B * D, x_sb=D, **dict(lnk, B=B))
            return x_new, h
        if shift is None:
            raise ValueError("the unfused-residual path fuses the last residual into the final layer instead")
        y = self._linear(a, w, key, gelu_in=gelu_in)
        x_new = torch.empty((n, B, D), dtype=BF16, device=self.device)
        h = N.ln_mod(x, shift, scale, x_st=x_st, x_sb=x_sb, y=y, gate=gate, x_out=x_new, **dict(lnk, B=B))
        return x_new, h

    def _linear(self, x, w: torch.Tensor, key: str, gelu_in: bool = False) -> torch.Tensor:
        """y = x w^T for a block projection (x [M, K] bf16 contiguous, or an fp8 operand pair (q, scale)
        that cp25_ln_mod_fp8 already produced). bf16: the own bf16 GEMM (GELU, if asked, applied in place to x
        first). fp8: row-quantised x (GELU fused) times the fp8 weight on cp25_gemm_fp8."""
        if isinstance(x, tuple):
            q, s = x
        elif self.linear_precision == "bf16":
            if gelu_in:
                N.gelu_(x)
            _require_gemm(w)
            return N.gemm_epi(x, w)
        else:
            q, s = N.quant_fp8_rows(x, gelu=gelu_in)
        self._own_fp8(w)
        w8, ws = self._fp8_weight(key, w)
        return N.gemm_fp8(q, s, w8, ws)

    # ---------------------------------------------------------------- loading
    def load_state_dict(self, state_dict: Dict[str, torch.Tensor], strict: bool = True) -> None:
        """Accepts the reference's checkpoint dict (`net.` prefix optional, `_extra_state` skipped,
        model_loader.py:173-174; text2world_model_rectified_flow.py:775-783)."""
        shapes = state_dict_shapes(self.cfg)
        sd = {}
        for k, v in state_dict.items():
            if k.startswith("net_ema."):
                continue
            k2 = k[4:] if k.startswith("net.") else k
            if k2.endswith("_extra_state"):
                continue
            if k2 in shapes:
                sd[k2] = v
        missing = [k for k in shapes if k not in sd]
        if missing and strict:
            raise KeyError(f"missing keys in DiT state dict: {missing[:8]}{'...' if len(missing) > 8 else ''}")
        cfg = self.cfg
        dev = self.device
        self.sd = {k: v.to(device=dev, dtype=shapes[k][1]).contiguous() for k, v in sd.items()}
        self._x_embed_w128 = None
        self._fp8_w = {}
        D = cfg.model_channels
        p = self.sd
        # fused / stacked views used by the hot path
        self.w_qkv = [torch.cat([p[f"blocks.{i}.self_attn.{n}_proj.weight"] for n in "qkv"], 0).contiguous()
                      for i in range(cfg.num_blocks)]
        for i in range(cfg.num_blocks):
            for n in "qkv":
                del p[f"blocks.{i}.self_attn.{n}_proj.weight"]  # keep only the fused copy in HBM
        self.w_ada1 = torch.cat([p[f"blocks.{i}.adaln_modulation_{m}.1.weight"]
                                 for i in range(cfg.num_blocks) for m in ("self_attn", "cross_attn", "mlp")], 0).float()
        self.w_ada2 = torch.stack([p[f"blocks.{i}.adaln_modulation_{m}.2.weight"]
                                   for i in range(cfg.num_blocks) for m in ("self_attn", "cross_attn", "mlp")], 0).float()
        self.w_final = p["final_layer.linear.weight"].float()
        if not cfg.use_wan_fp32_strategy:  # the bf16 final linear on the own GEMM: N padded with zero rows to 256
            wf = p["final_layer.linear.weight"]
            self.w_final_bf16 = torch.zeros(((wf.shape[0] + 255) // 256 * 256, D), dtype=BF16, device=dev)
            self.w_final_bf16[: wf.shape[0]] = wf
        # fp32 copies of the conditioning weights (the reference runs these layers under fp32 autocast)
        self.w_t1 = p["t_embedder.1.linear_1.weight"].float()
        self.w_t2 = p["t_embedder.1.linear_2.weight"].float()
        self.w_f1 = p["final_layer.adaln_modulation.1.weight"].float()
        self.w_f2 = p["final_layer.adaln_modulation.2.weight"].float()
        if cfg.cross_view_attn_map:  # the cross-view q|k|v projections as one [3D, D] GEMM per block
            self.w_cv_qkv = [torch.cat([p[f"blocks.{i}.cross_view_attn.{m}_proj.weight"] for m in "qkv"], 0).contiguous()
                             for i in range(cfg.num_blocks)]
        if cfg.adaln_view_embedding:
            self.w_view_proj = p["adaln_view_proj.weight"].float()
            self.b_view_proj = p["adaln_view_proj.bias"].float()
        self._bias_w = {}  # padded [w | bias | 0] copies for _bias_linear, per weight name
        self._embed_f32 = None  # multi-view patch embedding: fp32 weights padded to K % 32 == 0, view-channel fold
        self.refresh_norm_bounds()
        self._rope_cache.clear()
        if D % 512:
            raise ValueError("model_channels must be a multiple of 512")

    def refresh_norm_bounds(self) -> None:
        """Per-block (max|q|, max|k|) bounds for the attention softmax shift: the q/k RMSNorm (minimal_v4_dit.py:355-358)
        leaves every head row with |x| <= sqrt(hd) * max|weight|, RoPE is a rotation; 2 % covers the two bf16
        roundings. One host read per weight, at load time (call again after changing a q/k norm weight). The
        library picks the shift mode from them (a fixed shift where the product allows, else an online max)."""
        cfg, p = self.cfg, self.sd
        hd = cfg.head_dim

        def nb(w: torch.Tensor) -> float:
            return float(w.float().abs().max()) * hd ** 0.5 * 1.02

        self.attn_bounds = [(nb(p[f"blocks.{i}.self_attn.q_norm.weight"]), nb(p[f"blocks.{i}.self_attn.k_norm.weight"]))
                            for i in range(cfg.num_blocks)]
        self.xattn_bounds = [(nb(p[f"blocks.{i}.cross_attn.q_norm.weight"]),
                              nb(p[f"blocks.{i}.cross_attn.k_norm.weight"])) for i in range(cfg.num_blocks)]
        if cfg.cross_view_attn_map:
            self.cvattn_bounds = [(nb(p[f"blocks.{i}.cross_view_attn.q_norm.weight"]),
                                   nb(p[f"blocks.{i}.cross_view_attn.k_norm.weight"])) for i in range(cfg.num_blocks)]

    def attention_kernels(self, L: int) -> Dict[str, str]:
        """The attention kernel forms block 0 launches at L tokens (self) and against the text context (cross)."""
        hd = self.cfg.head_dim
        out = {}
        for name, bounds, lk in (("self", self.attn_bounds[0], L), ("cross", self.xattn_bounds[0], 512)):
            _, kw = self._attn_mode(bounds, hd)
            fp8 = 0
            if name == "self" and kw.get("prescaled") and self.attention_precision != "bf16":
                qb, kb = kw["norm_bounds"]
                fp8 = 0 if qb * kb > 60.0 else (2 if self.attention_precision == "fp8" and 1.13 * qb * kb <= 30.0 else 1)
            pre = kw.get("prescaled", False)
            if name == "self" and self._k_slots(kw) is not None and self.cp_group is None:
                pre = 2
            out[name] = N.attn_kernel_name(lk, kw.get("softmax_scale"), kw["norm_bounds"], pre, fp8)
        return out

    def state_dict_keys(self) -> List[str]:
        return list(state_dict_shapes(self.cfg).keys())

    # ---------------------------------------------------------------- context parallel
    def enable_context_parallel(self, process_group) -> None:
        self.cp_group = process_group

    def disable_context_parallel(self) -> None:
        self.cp_group = None

    @property
    def is_context_parallel_enabled(self) -> bool:
        return self.cp_group is not None

    # ---------------------------------------------------------------- per-prompt constants
    @torch.no_grad()
    def prepare_context(self, crossattn_emb: torch.Tensor) -> ContextCache:
        """crossattn_emb [B, Lctx, proj_in] -> per-block cross-attention K/V (normed)."""
        cfg = self.cfg
        p = self.sd
        B, Lc, c_in = crossattn_emb.shape
        if cfg.use_crossattn_projection:
            # crossattn_proj = Linear + bias + exact GELU (minimal_v4_dit.py:1430-1434, applied at :1604); EPI_GELU
            # applies the GELU to the rounded sum (cp25_gelu's arithmetic)
            ctx = self._bias_linear(crossattn_emb.reshape(B * Lc, c_in), "crossattn_proj.0", N.EPI_GELU)
        else:
            ctx = crossattn_emb.to(device=self.device, dtype=BF16).reshape(B * Lc, c_in).contiguous()
        H, hd = cfg.num_heads, cfg.head_dim
        ks, vs = [], []
        for i in range(cfg.num_blocks):
            # cross-attention k/v projections (minimal_v4_dit.py:401-404) of the text context, once per prompt
            wk, wv = p[f"blocks.{i}.cross_attn.k_proj.weight"], p[f"blocks.{i}.cross_attn.v_proj.weight"]
            _require_gemm(wk, "cross-attention k_proj")
            _require_gemm(wv, "cross-attention v_proj")
            k = N.gemm_epi(ctx, wk)
            N.head_rmsnorm_rope(k, n_rows=B * Lc, B=1, H=H, head_off=0,
                                weight=p[f"blocks.{i}.cross_attn.k_norm.weight"])
            v = N.gemm_epi(ctx, wv)
            ks.append(k.view(B, Lc, H, hd))
            vs.append(v.view(B, Lc, H, hd))
        return ContextCache(B=B, k=ks, v=vs)

    def _bias_linear(self, x: torch.Tensor, key: str, epilogue: int = 0) -> Optional[torch.Tensor]:
        """bf16 nn.Linear with bias (weight / bias `key`.weight / .bias) of x [M, K] on the hand-written GEMM: the bias
        rides as one more K column (a' = [x | 1 | 0..], w' = [w | bias | 0..], K padded to a multiple of 64), so it
        enters the fp32 accumulator before the product's one bf16 rounding, as the library's bias epilogue adds it
        (tests/test_gemm_f32_gpu.py: within 1 bf16 ulp of F.linear(bias), the two sum in different orders). ValueError
        where the GEMM is not built for the shape. The padded weight replaces the state dict's weight (which becomes a
        view of it), so the net holds one copy; the padded operand is a copy of x (for crossattn_proj: [B * 512,
        100 416] bf16, ~0.2 GB, once per prompt, freed on return)."""
        p = self.sd
        w, bias = p[key + ".weight"], p[key + ".bias"]
        n_out, k_in = w.shape
        kp = (k_in + 1 + 63) // 64 * 64
        if not N.gemm_supported(n_out, kp):
            raise ValueError(f"{key}: [{n_out}, {k_in}] + bias is not a shape the own GEMM is built for "
                             "(N a multiple of 256)")
        wb = self._bias_w.get(key)
        if wb is None:
            wb = torch.zeros((n_out, kp), dtype=BF16, device=self.device)
            wb[:, :k_in] = w
            wb[:, k_in] = bias
            self._bias_w[key] = wb
            p[key + ".weight"] = wb[:, :k_in]  # one copy in HBM: the state dict's weight is now a view of wb
        a = torch.empty((x.shape[0], kp), dtype=BF16, device=self.device)
        a[:, :k_in] = x
        a[:, k_in] = 1.0
        a[:, k_in + 1:] = 0.0  # only the pad columns are cleared (no full-size zero fill)
        return N.gemm_epi(a, wb, epilogue=epilogue)

    def rope_tables(self, geo: Geometry) -> Tuple[torch.Tensor, torch.Tensor]:
        """cos/sin [n_tok, 64] of this shard; multi-view: every view's positions restart at t = 0
        (MultiCameraVideoRopePosition3DEmb.generate_embeddings, multiview_dit.py:108-130)."""
        key = (geo.T, geo.Hp, geo.Wp, geo.n_views)
        if key not in self._rope_cache:
            fr = rope_freqs(self.cfg, geo.T_view, geo.Hp, geo.Wp, self.sd, self.device)[:, :64]
            fr = fr.repeat(geo.n_views, 1).contiguous()
            self._rope_cache[key] = (torch.cos(fr).contiguous(), torch.sin(fr).contiguous())
        c, s = self._rope_cache[key]
        if geo.frames is not None:  # a frame-sharded rank: its tokens' rows
            idx = geo.token_ids(self.device)
            return c[idx], s[idx]
        return c[geo.tok0: geo.tok0 + geo.n_tok], s[geo.tok0: geo.tok0 + geo.n_tok]

    # ---------------------------------------------------------------- fp32 conditioning
    @torch.no_grad()
    def action_embedding(self, action: torch.Tensor, B: int, T: int):
        """Action-conditioned nets: action [B' (1 or B), A, action_dim] -> (emb_D [B, T|1, D],
        emb_3D [B, T|1, 3D]) bf16, the reference's bf16 Mlp (fc1 + bias, GELU tanh, fc2 + bias)
        (action_conditioned_minimal_v1_lvg_dit.py:28-45, per-chunk :104-107, per-latent-frame
        :257-270 with a zero embedding for latent frame 0)."""
        cfg = self.cfg
        p = self.sd
        a = action.to(device=self.device, dtype=BF16)
        Ba, A, dim = a.shape
        if dim != cfg.action_dim:
            raise ValueError(f"action_dim {dim} != the net's {cfg.action_dim}")
        if cfg.action_per_latent_frame:
            per = cfg.action_per_latent_frame
            if A % per or A // per + 1 != T:
                raise ValueError(f"{A} actions do not give {T - 1} latent frames of {per}")
            a = a.reshape(Ba, A // per, per * dim)
        else:
            if A != cfg.num_action_per_chunk:
                raise ValueError(f"{A} actions, the net takes {cfg.num_action_per_chunk} per chunk")
            a = a.reshape(Ba, 1, A * dim)

        def mlp(name):  # fc1 and fc2 (+ bias) on the hand-written GEMM, the tanh GELU between them in torch
            h = self._bias_linear(a.reshape(-1, a.shape[-1]), name + ".fc1")
            h = F.gelu(h, approximate="tanh")
            y = self._bias_linear(h, name + ".fc2")
            return y.view(*a.shape[:-1], -1)

        e_d, e_3d = mlp("action_embedder_B_D"), mlp("action_embedder_B_3D")
        if cfg.action_per_latent_frame:
            e_d = torch.cat([torch.zeros_like(e_d[:, :1]), e_d], 1)
            e_3d = torch.cat([torch.zeros_like(e_3d[:, :1]), e_3d], 1)
        if Ba != B:
            e_d, e_3d = e_d.expand(B, -1, -1), e_3d.expand(B, -1, -1)
        return e_d, e_3d

    @torch.no_grad()
    def scale_timesteps(self, t: torch.Tensor) -> torch.Tensor:
        """The net's `timesteps_B_T * self.timestep_scale` (minimal_v1_lvg_dit.py:49, multiview_dit.py:535) of the
        sampler's fp32 timesteps, as fp32 values for forward_tokens. use_wan_fp32_strategy nets: in fp32. The others
        (the multi-view nets, predict2_multiview/configs/vid2vid/defaults/net.py:52,105) take t in the net's dtype:
        bf16(bf16(t) * scale). The reference's rectified-flow denoise hands these nets fp32 timesteps
        (video2world_model_rectified_flow.py:113-127), which the bf16 t-embedder cannot take without the fp32
        autocast the flag turns off (TimestepEmbedding.linear_1, minimal_v4_dit.py:776, would raise on an fp32 input
        against its bf16 weight); its EDM denoise casts them to the net dtype exactly when the flag is off
        (video2world_model.py:231-236), and that is the cast restated here."""
        t = t.to(self.device).float()
        if self.cfg.use_wan_fp32_strategy:
            return t * self.cfg.timestep_scale
        return (t.to(BF16) * self.cfg.timestep_scale).float()

    def _sincos(self, t_B_T: torch.Tensor) -> torch.Tensor:
        """Timesteps (minimal_v4_dit.py:727-747): [cos | sin] of t * 10000^(-i / half) in fp32 -> [B, T, D] fp32."""
        D = self.cfg.model_channels
        B, T = t_B_T.shape
        half = D // 2
        expo = -math.log(10000) * torch.arange(half, dtype=F32, device=self.device)
        expo = expo / (half - 0.0)
        arg = t_B_T.flatten().float()[:, None] * torch.exp(expo)[None, :]
        return torch.cat([torch.cos(arg), torch.sin(arg)], dim=-1).view(B, T, D)

    def time_modulation(self, t_B_T: torch.Tensor, action: Optional[torch.Tensor] = None):
        """t (scale_timesteps) [B, T] fp32 -> (block mods bf16 [nb, 3, B, T, 3D], final shift / scale [B, T, D] each:
        fp32 under use_wan_fp32_strategy, else bf16). fp32 math (use_wan_fp32_strategy), else _time_modulation_bf16.
        Action nets add the action embeddings to the embedding and the AdaLN-LoRA term before the norm
        (action_conditioned_minimal_v1_lvg_dit.py:298-305)."""
        cfg = self.cfg
        if not cfg.use_wan_fp32_strategy:
            return self._time_modulation_bf16(t_B_T, action)
        p = self.sd
        D = cfg.model_channels
        B, T = t_B_T.shape
        sincos = self._sincos(t_B_T)
        # every fp32 linear below on cp25_gemm_f32 (fp32 MFMA): TimestepEmbedding (minimal_v4_dit.py:727-788)
        h = N.gemm_f32(sincos.view(B * T, D), self.w_t1, act=N.ACT_SILU)
        lora = N.gemm_f32(h, self.w_t2).view(B, T, 3 * D)
        if cfg.action_dim:
            if action is None:
                raise ValueError("this action-conditioned net needs `action`")
            e_d, e_3d = self.action_embedding(action, B, T)
            sincos = sincos + e_d.float()
            lora = lora + e_3d.float()
        elif action is not None:
            raise ValueError("`action` given to a net without action embedders")
        xf = sincos
        emb = ((xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6)) * p["t_embedding_norm.weight"].float())
        se = F.silu(emb)  # [B, T, D]
        nb3 = 3 * cfg.num_blocks
        se = se.reshape(B * T, D)
        lora2 = lora.view(B * T, 3 * D)
        # AdaLN-LoRA of every block sub-layer (minimal_v4_dit.py:1136-1154): the 3 nb Linear(D, A) as one GEMM, the
        # 3 nb Linear(A, 3D) as one batched GEMM over the column blocks of its output, + the LoRA term in the epilogue
        a1 = N.gemm_f32(se, self.w_ada1).view(B * T, nb3, -1).transpose(0, 1)  # [nb3, BT, A]
        a2 = N.gemm_f32(a1, self.w_ada2, add=lora2)  # [nb3, BT, 3D]
        mods = a2.view(cfg.num_blocks, 3, B, T, 3 * D).to(BF16)
        f1 = N.gemm_f32(se, self.w_f1)
        f2 = N.gemm_f32(f1, self.w_f2, add=lora2[:, : 2 * D]).view(B, T, 2 * D)
        shift_f, scale_f = f2.chunk(2, dim=-1)
        return mods, shift_f, scale_f

    def _time_modulation_bf16(self, t_B_T: torch.Tensor, action: Optional[torch.Tensor] = None):
        """time_modulation of a net with use_wan_fp32_strategy=False: the same layers without the fp32 autocast
        (multiview_dit.py:544-548 / multiview_cross_dit.py:823-827, minimal_v4_dit.py:1136-1154 AdaLN, :974-995 final
        layer), i.e. in the net's bf16. Every linear is a bf16 GEMM (bf16 operands, fp32 accumulation, one bf16
        rounding: cp25_gemm_f32 on the bf16 values, rounded), every elementwise op one bf16 torch op: the sinusoid
        rounded to bf16, SiLU on the rounded linear_1 output, TE RMSNorm (fp32 math, one rounding), the AdaLN-LoRA
        sum `modulation(emb) + lora` of two bf16 tensors. Returns bf16 shift / scale for the final layer."""
        cfg = self.cfg
        D = cfg.model_channels
        B, T = t_B_T.shape

        def lin(x, w, **kw):  # bf16 nn.Linear (no bias) of bf16 x on the fp32 MFMA GEMM, one rounding
            return N.gemm_f32(x.float(), w, **kw).to(BF16)

        sincos = self._sincos(t_B_T).to(BF16).view(B * T, D)
        h = F.silu(lin(sincos, self.w_t1))
        lora = lin(h, self.w_t2)  # [BT, 3D]
        if cfg.action_dim:
            if action is None:
                raise ValueError("this action-conditioned net needs `action`")
            e_d, e_3d = self.action_embedding(action, B, T)  # [B, T or 1, *]: broadcast over the frames
            sincos = (sincos.view(B, T, D) + e_d).reshape(B * T, D)
            lora = (lora.view(B, T, 3 * D) + e_3d).reshape(B * T, 3 * D)
        elif action is not None:
            raise ValueError("`action` given to a net without action embedders")
        xf = sincos.float()
        emb = ((xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6)) * self.sd["t_embedding_norm.weight"].float())
        se = F.silu(emb.to(BF16))  # [BT, D] bf16
        nb3 = 3 * cfg.num_blocks
        a1 = lin(se, self.w_ada1).view(B * T, nb3, -1).transpose(0, 1)  # [nb3, BT, A]
        a2 = lin(a1, self.w_ada2)  # [nb3, BT, 3D]
        mods = (a2 + lora[None]).view(cfg.num_blocks, 3, B, T, 3 * D)
        f2 = lin(lin(se, self.w_f1), self.w_f2) + lora[:, : 2 * D]
        shift_f, scale_f = f2.view(B, T, 2 * D).chunk(2, dim=-1)
        return mods, shift_f, scale_f

    # ---------------------------------------------------------------- hot path
    @torch.no_grad()
    def n_views_for(self, T: int) -> int:
        """Views stacked along the latent T axis (multi-view nets: T / state_t, MultiViewDiT :461)."""
        cfg = self.cfg
        if not cfg.n_cameras_emb:
            return 1
        if cfg.state_t <= 0 or T % cfg.state_t:
            raise ValueError(f"{T} latent frames are not a whole number of {cfg.state_t}-frame views")
        return T // cfg.state_t

    def embed_patches(self, patch_rows: torch.Tensor, geo: Geometry,
                      view_indices: Optional[torch.Tensor] = None, rows_k128: bool = False) -> torch.Tensor:
        """x_embedder (PatchEmbed Linear, minimal_v4_dit.py:846-913) of [n, Bx, 72] patch rows -> [n, Bx, D].
        rows_k128: the caller made patch_rows with patchify(ld=128), i.e. they are the [:, :72] view of a [n, 128]
        buffer whose columns 72.. the kernel zeroed; the own GEMM then multiplies the whole padded rows (K = 128).
        Multi-view nets also concatenate a view embedding as input channels
        (prepare_embedded_sequence, multiview_dit.py:462-490); those channels are constant over a view, so
        their patch features (c, p1, p2) fold into one per-view bias: y = rows W72^T + e_v Wv^T, summed
        in fp32 and rounded once to bf16 like the reference's single bf16 GEMM."""
        cfg = self.cfg
        p = self.sd
        D = cfg.model_channels
        n, Bx, f = patch_rows.shape
        w = p["x_embedder.proj.1.weight"]
        if not cfg.view_condition_dim:
            if rows_k128 and (Bx != 1 or f != 72 or patch_rows.stride(0) != 128 or patch_rows.stride(2) != 1):
                raise ValueError("rows_k128: expected the [n, 1, 72] view of patchify(ld=128)'s [n, 128] buffer")
            if f > 128 or not N.gemm_supported(D, 128):
                raise ValueError(f"x_embedder [{D}, {f}]: the own GEMM takes f <= 128 features and D % 256 == 0")
            # the zero-padded K = 128 operand of the own GEMM against the weight zero-padded to 128 columns (the same
            # sums as K = 72): rows from patchify(ld=128) are that operand already, other rows are copied into it
            if rows_k128:
                a = torch.as_strided(patch_rows, (n, 128), (128, 1))
            else:
                a = torch.zeros((n * Bx, 128), dtype=BF16, device=self.device)
                a[:, :f] = patch_rows.reshape(n * Bx, f)
            wp = self._x_embed_w128
            if wp is None or wp.shape[0] != D:
                wp = torch.zeros((D, 128), dtype=BF16, device=self.device)
                wp[:, :f] = w[:, :f]
                self._x_embed_w128 = wp
            return N.gemm_epi(a, wp).view(n, Bx, D)
        V = geo.n_views
        if view_indices is None:
            view_indices = torch.arange(V, device=self.device)
        view_indices = view_indices.to(self.device).long().clamp(max=cfg.n_cameras_emb - 1)
        vdim = cfg.view_condition_dim
        kf, kv = -(-f // 32) * 32, -(-vdim // 32) * 32  # cp25_gemm_f32 takes K % 32 == 0
        if self._embed_f32 is None or self._embed_f32[0].shape[1] != kf:
            # fp32 weights zero-padded to K = kf (patch features: 96 for the 72 of the 2B layout) and kv (the view
            # channels folded over (p1, p2, t))
            wk = torch.zeros((D, kf), dtype=F32, device=self.device)
            wk[:, :f] = w[:, :f]
            wv = torch.zeros((D, kv), dtype=F32, device=self.device)
            wv[:, :vdim] = w[:, f:].float().view(D, vdim, -1).sum(-1)
            self._embed_f32 = (wk, wv)
        wk, wv = self._embed_f32
        emb = torch.zeros((V, kv), dtype=F32, device=self.device)
        emb[:, :vdim] = p["view_embeddings.weight"][view_indices]
        bias = N.gemm_f32(emb, wv)  # [V, D]
        view_of_tok = torch.arange(geo.tok0, geo.tok0 + n, device=self.device) // geo.L_view
        rows = torch.zeros((n, Bx, kf), dtype=F32, device=self.device)
        rows[:, :, :f] = patch_rows
        # y[b] = rows[:, b] wk^T + bias[view of the token], batched over the Bx entries; fp32, rounded once
        y = torch.empty((n, Bx, D), dtype=F32, device=self.device)
        N.gemm_f32(rows.transpose(0, 1), wk.expand(Bx, D, kf), add=bias[view_of_tok].expand(Bx, n, D),
                   out=y.transpose(0, 1), split_k=False)
        return y.to(BF16)

    def forward_tokens(self, patch_rows: torch.Tensor, t_B_T: torch.Tensor, ctx: ContextCache,
                       geo: Geometry, action: Optional[torch.Tensor] = None,
                       view_indices: Optional[torch.Tensor] = None, shared_batch: bool = False,
                       rows_k128: bool = False) -> torch.Tensor:
        """patch_rows: [n_tok, Bx, 72] bf16 (Bx = 1 shares the input across the CFG batch; rows_k128: made by
        patchify(ld=128), see embed_patches);
        t_B_T: [B, T] fp32, already scaled. Returns the final layer output [n_tok, B, 64] fp32
        (feature order (p1 p2 C) = patch layout). shared_batch: the caller guarantees every batch entry
        has the same t (and action), so with Bx = 1 they differ only in the text context (_blocks).

        CP = 1: one pass over the batch (B = 2 = [cond, uncond]).
        CP > 1: the batch entries run as two software-pipelined lanes on the current stream: each
        lane yields right after queueing its block's asynchronous RCCL K/V all-gather, and the other
        lane's whole block is issued before the first lane waits for it, so each transfer runs
        behind a lane-block of compute (one stream: no cross-stream hazards; a two-stream variant
        that also ran the lanes' kernels concurrently hung intermittently in device synchronisation
        on MI355X and was dropped)."""
        cfg = self.cfg
        p = self.sd
        B = ctx.B
        D = cfg.model_channels
        n = geo.n_tok
        Bx = patch_rows.shape[1]
        x_in = self.embed_patches(patch_rows, geo, view_indices, rows_k128=rows_k128)
        mods, shift_f, scale_f = self.time_modulation(t_B_T, action)
        cos, sin = self.rope_tables(geo)
        sharded = geo.frames is not None
        if sharded:
            if not cfg.cross_view_attn_map:
                raise ValueError("a frame-sharded geometry is the cross-view nets' CP layout")
            # the rank's frames of the per-frame modulation, then everything below on the local geometry
            fidx = torch.tensor(geo.frames, device=self.device)
            mods, shift_f, scale_f = mods[:, :, :, fidx], shift_f[:, fidx], scale_f[:, fidx]
            geo = geo.local()
        if cfg.adaln_view_embedding:
            mods = self._view_modulation(mods, geo, view_indices)
        cp = self.cp_group
        cp_size = 1 if cp is None else torch.distributed.get_world_size(cp)
        cv = None
        if cfg.cross_view_attn_map:
            if geo.n_tok != geo.L or (cp_size > 1 and not sharded):
                raise ValueError("cross-view nets shard by frame under context parallelism (Geometry.frame_shard)")
            cv = self._cross_view_neighbours(geo, view_indices)
        if B == 1 or (cp_size == 1 and not self.force_lanes) or (cv is not None and cp_size == 1):
            gen = self._blocks(x_in, mods, shift_f, scale_f, ctx, geo, cos, sin, cp, cp_size, shared_batch,
                               cv_nbrs=cv)
            while True:
                try:
                    next(gen)
                except StopIteration as e:
                    return e.value
        if cv is not None:  # per-view self-attention gathers each view's frames; no shared block-0 prefix
            lanes = [self._blocks(x_in[:, (0 if Bx == 1 else b):(0 if Bx == 1 else b) + 1], mods[:, :, b:b + 1],
                                  shift_f[b:b + 1], scale_f[b:b + 1],
                                  ContextCache(B=1, k=[t[b:b + 1] for t in ctx.k], v=[t[b:b + 1] for t in ctx.v]), geo,
                                  cos, sin, cp, cp_size, cv_nbrs=cv) for b in range(B)]
            return torch.cat(run_lanes(lanes), dim=1)
        if B == 1 or (cp_size == 1 and not self.force_lanes):
            gen = self._blocks(x_in, mods, shift_f, scale_f, ctx, geo, cos, sin, cp, cp_size, shared_batch)
            while True:
                try:
                    next(gen)
                except StopIteration as e:
                    return e.value
        lanes = []
        prefix = None
        if shared_batch and Bx == 1 and self.share_cfg_block0:
            # the entries' identical block-0 prefix once (its K/V gather waited on in place), then the lanes
            cb = ContextCache(B=1, k=[t[:1] for t in ctx.k], v=[t[:1] for t in ctx.v])
            gen = self._blocks(x_in, mods[:, :, :1], shift_f[:1], scale_f[:1], cb, geo, cos, sin, cp, cp_size,
                               prefix_only=True)
            while prefix is None:
                try:
                    next(gen)
                except StopIteration as e:
                    prefix = e.value
        for b in range(B):
            cb = ContextCache(B=1, k=[t[b:b + 1] for t in ctx.k], v=[t[b:b + 1] for t in ctx.v])
            xb = x_in[:, (0 if Bx == 1 else b):(0 if Bx == 1 else b) + 1]
            lanes.append(self._blocks(xb, mods[:, :, b:b + 1], shift_f[b:b + 1], scale_f[b:b + 1], cb, geo, cos,
                                      sin, cp, cp_size, prefix=prefix))
        return torch.cat(run_lanes(lanes), dim=1)

    def _view_modulation(self, mods: torch.Tensor, geo: Geometry, view_indices: Optional[torch.Tensor]) -> torch.Tensor:
        """Cross-view nets' AdaLN view embedding (multiview_cross_dit.py:807-813, 355-404): adaln_view_proj(
        adaln_view_embedder(view id)) [V, 9D] (cp25_gemm_f32 with the bias as addend, rounded to bf16: the fp32-autocast
        linear, or with use_wan_fp32_strategy=False the bf16 linear, whose bf16 operands make the same sums) in the chunk order
        (shift, scale, gate) x (self-attn, cross-attn, mlp), rounded to bf16 and added to the bf16 modulation of every
        frame of the view (one bf16 rounding, the reference's `m + view_m.type_as(x)`)."""
        cfg, D, V = self.cfg, self.cfg.model_channels, geo.n_views
        ids = self._view_ids(geo, view_indices)
        e = self.sd["adaln_view_embedder.weight"][ids].float()
        # (the same sums either way: bf16 e, w and bias, fp32 accumulation with the bias, one rounding to bf16)
        vp = N.gemm_f32(e, self.w_view_proj, add=self.b_view_proj).to(BF16).view(V, 3, 3 * D)
        per_frame = vp.repeat_interleave(geo.T_view, dim=0)  # [T, 3, 3D]: frame t belongs to view t // T_view
        if mods.shape[3] != per_frame.shape[0]:
            raise ValueError(f"modulation has {mods.shape[3]} frames, the views {per_frame.shape[0]}")
        return mods + per_frame.permute(1, 0, 2)[None, :, None]

    def _view_ids(self, geo: Geometry, view_indices: Optional[torch.Tensor]) -> torch.Tensor:
        V = geo.n_views
        ids = torch.arange(V, device=self.device) if view_indices is None else view_indices.to(self.device).long()
        if ids.numel() != V:
            raise ValueError(f"{ids.numel()} view indices for {V} views")
        return ids.clamp(max=self.cfg.n_cameras_emb - 1)

    def _cross_view_neighbours(self, geo: Geometry, view_indices: Optional[torch.Tensor]) -> List[List[int]]:
        """Per view position: the positions of its neighbour views present in the input, in the reference's key order
        (CrossViewAttention.forward, multiview_cross_dit.py:160-186: neighbour ids of the view's id looked up among the
        input's view ids, absent ones dropped -- the reference masks them -- positions sorted descending)."""
        ids = self._view_ids(geo, view_indices).tolist()
        amap = self.cfg.cross_view_attn_map
        pos = {v: i for i, v in enumerate(ids)}
        return [sorted((pos[u] for u in amap[v] if u in pos), reverse=True) if v < len(amap) else [] for v in ids]

    def _per_view_attention(self, q, k, v, o, geo: Geometry, attn_kw: dict) -> None:
        """Self-attention of each view over its own tokens ([B, n, H, hd] views, views contiguous along n): the
        cross-view net's per-view self-attention (multiview_cross_dit.py:425-435, "(b v) (t h w)"). A q normalised in
        the kernel reads the view's rows of the RoPE tables (positions restart per view)."""
        if "fp8_qk" in attn_kw:
            raise NotImplementedError("the fp8 attention forms are not built for per-view self-attention")
        Lv = geo.L_view
        for vi in range(geo.n_views):
            sl = slice(vi * Lv, (vi + 1) * Lv)
            kw = attn_kw
            qn = attn_kw.get("q_norm")
            if qn is not None and qn.get("cos") is not None:
                kw = dict(attn_kw, q_norm=dict(qn, cos=qn["cos"][sl], sin=qn["sin"][sl]))
            N.attn_fwd(q[:, sl], k[:, sl], v[:, sl], out=o[:, sl], **kw)

    def _cross_view(self, i: int, x: torch.Tensor, B: int, geo: Geometry, nbrs: List[List[int]], mods_i1: torch.Tensor,
                    lnk: dict, shift, scale):
        """The cross-view sub-layer of MultiViewCrossBlock (multiview_cross_dit.py:436-450 over CrossViewAttention
        :138-228): x + output_proj(attention of every view's tokens, per latent frame, to its neighbours' tokens of the
        same frame) on the affine-LayerNormed x, un-gated; then the text cross-attention's LN-mod (shift, scale).
        q / k / v come from one [3D, D] GEMM over all tokens (a neighbour's k / v rows are its own projections; the
        reference projects the gathered neighbour rows, the same rows), q / k RMS-normed per head (no RoPE), and the
        neighbours' K / V rows of each view gathered into one key sequence per frame. A view with no neighbour present
        adds nothing (the reference would attend over an all-masked row). Returns (x', h)."""
        cfg, p = self.cfg, self.sd
        D, H, hd = cfg.model_channels, cfg.num_heads, cfg.head_dim
        pre = f"blocks.{i}."
        n, V, Tv, hw = geo.n_tok, geo.n_views, geo.T_view, geo.hw
        hv = N.layer_norm(x.view(n * B, D), p[pre + "layer_norm_cross_view_attn.weight"],
                          p[pre + "layer_norm_cross_view_attn.bias"])
        w = self.w_cv_qkv[i]
        _require_gemm(w, "cross-view q|k|v")
        qkv = N.gemm_epi(hv, w)
        q_scale, attn_kw = self._attn_mode(self.cvattn_bounds[i], hd)
        N.head_rmsnorm_rope(qkv, n_rows=n * B, B=B, H=H, head_off=0, weight=p[pre + "cross_view_attn.q_norm.weight"],
                            out_scale=q_scale)
        N.head_rmsnorm_rope(qkv, n_rows=n * B, B=B, H=H, head_off=D, weight=p[pre + "cross_view_attn.k_norm.weight"])
        q5 = qkv.view(V, Tv, hw, B, 3 * D)
        o = torch.zeros((n, B, D), dtype=BF16, device=self.device)
        o5 = o.view(V, Tv, hw, B, D)
        for vi in range(V):
            if not nbrs[vi]:
                continue
            # [Tv, n_nbr * hw, B, 2D]: frame t's key sequence = the neighbours' rows of frame t, in nbrs order
            kv = torch.stack([q5[u, :, :, :, D:] for u in nbrs[vi]], dim=1).reshape(Tv, len(nbrs[vi]) * hw, B, 2 * D)
            for b in range(B):
                N.attn_fwd(q5[vi, :, :, b, :D].unflatten(-1, (H, hd)), kv[:, :, b, :D].unflatten(-1, (H, hd)),
                           kv[:, :, b, D:].unflatten(-1, (H, hd)), out=o5[vi, :, :, b].unflatten(-1, (H, hd)), **attn_kw)
        gate1 = torch.ones_like(mods_i1)[..., :D]  # the residual is not gated: bf16(1 * y) = y
        return self._proj_res(o.view(n * B, D), p[pre + "cross_view_attn.output_proj.weight"],
                              pre + "cross_view_attn.output_proj", x, B * D, D, gate1, B, geo, n, lnk, shift, scale)

    def _blocks(self, x_in, mods, shift_f, scale_f, ctx: ContextCache, geo: Geometry, cos, sin, cp, cp_size,
                shared_batch: bool = False, prefix=None, prefix_only: bool = False, cv_nbrs=None):
        """Generator: issues the 28 blocks + final layer for the batch entries in x_in/mods/ctx on the
        current stream; returns the final layer output [n, B, 64] fp32. Yields (so the caller can
        issue the other lane) right after each self-attention K/V gather is queued (CP > 1), or after
        each block (CP = 1).

        shared_batch (the CFG pair: one input x, one t, one action, only the text context differs): block
        0's self-attention sub-layer and its residual, and the cross-attention query, see identical
        inputs in every batch entry, so they run once (B = 1) and the cross-attention reads that query
        with batch stride 0 against each entry's own text K/V. Every later sub-layer has per-entry
        inputs. Same values as running both entries (tests/test_dit_gpu.py::test_shared_cfg_block0).
        CP lanes (one entry each) share it the same way: prefix_only=True runs block 0 up to the cross-attention
        LN-mod for one entry and returns (x, h); each lane then starts from prefix=(x, h)."""
        cfg = self.cfg
        p = self.sd
        B = ctx.B
        D, H, hd = cfg.model_channels, cfg.num_heads, cfg.head_dim
        n = geo.n_tok
        Bx = x_in.shape[1]
        share0 = (shared_batch and Bx == 1 and B > 1 and (cp is None or cp_size == 1) and self.share_cfg_block0
                  and cv_nbrs is None)

        def mod(i, j, nb=None):  # (shift, scale, gate) bf16 [B, T, D] views of block i, sub-layer j (first nb)
            m = mods[i, j] if nb is None else mods[i, j][:nb]
            return m[..., :D], m[..., D:2 * D], m[..., 2 * D:]

        # fp8: each LN-mod emits its h straight as the next GEMM's fp8 operand (q, scale)
        common = dict(n_tok=n, B=B, tok0=geo.tok0, hw=geo.hw)
        lnk = dict(common, fp8=self.linear_precision == "fp8")
        lnk1 = dict(lnk, B=1)
        if prefix is None:
            sh, sc, _ = mod(0, 0, 1 if share0 else None)
            x = x_in
            h = N.ln_mod(x, sh, sc, x_st=x_in.stride(0), x_sb=0 if Bx == 1 else x_in.stride(1),
                         **(lnk1 if share0 else lnk))
        else:
            x, h = prefix
        y = None
        gate_prev = None
        for i in range(cfg.num_blocks):
            pre = f"blocks.{i}."
            Bs = 1 if (share0 and i == 0) else B  # batch rows up to the cross-attention query
            if prefix is not None and i == 0:
                pass  # block 0 up to here ran once for every lane (prefix)
            else:
                # ---- self attention
                o = torch.empty((n, Bs, D), dtype=BF16, device=self.device)
                ev = None
                if self.attn_events is not None:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                if cp is None or cp_size == 1:
                    q_scale, attn_kw = self._self_attn_mode(i, hd)
                    kslots = self._k_slots(attn_kw)
                    qkv = self._qkv_k_normed(h, i, n * Bs, Bs, cos, sin, kslots)  # [n*Bs, 3D], k normed + roped
                    if self._q_norm_in_attention(attn_kw):
                        attn_kw = dict(attn_kw, q_norm=dict(weight=p[pre + "self_attn.q_norm.weight"], cos=cos, sin=sin,
                                                            out_scale=q_scale))
                    else:
                        N.head_rmsnorm_rope(qkv, n_rows=n * Bs, B=Bs, H=H, head_off=0,
                                            weight=p[pre + "self_attn.q_norm.weight"], cos=cos, sin=sin,
                                            out_scale=q_scale)
                    if kslots is not None:
                        attn_kw = dict(attn_kw, k_norm_slots=kslots)
                    q = qkv.view(n, Bs, 3 * D)[:, :, :D].view(n, Bs, H, hd).transpose(0, 1)
                    kk = qkv.view(n, Bs, 3 * D)[:, :, D:2 * D].view(n, Bs, H, hd).transpose(0, 1)
                    vv = qkv.view(n, Bs, 3 * D)[:, :, 2 * D:].view(n, Bs, H, hd).transpose(0, 1)
                    attn_kw = self._fp8_qk(qkv[:, :D], qkv[:, D:2 * D], Bs, H, hd, attn_kw, vv)
                    if ev is not None:
                        ev[0].record()
                    if cv_nbrs is not None:
                        self._per_view_attention(q, kk, vv, o.view(n, Bs, H, hd).transpose(0, 1), geo, attn_kw)
                    else:
                        N.attn_fwd(q, kk, vv, out=o.view(n, Bs, H, hd).transpose(0, 1), **attn_kw)
                    lk = kk.shape[1] if cv_nbrs is None else geo.L_view
                else:
                    yield from self._cp_self_attention(i, h, o, cos, sin, n, B, cp, cp_size,
                                                       ev[0] if ev is not None else None,
                                                       views=geo if cv_nbrs is not None else None)
                    lk = cp_size * (n if cv_nbrs is None else geo.L_view)
                if ev is not None:
                    ev[1].record()
                    self.attn_events.append((ev[0], ev[1], 4.0 * Bs * H * n * lk * hd))
                # ---- x += g_sa * (o W_o^T) ; LN-mod for cross attention
                nb = 1 if Bs == 1 and B > 1 else None
                _, _, g_sa = mod(i, 0, nb)
                sh, sc, _ = mod(i, 1, nb)
                if i == 0:
                    x_st, x_sb = x_in.stride(0), (0 if Bx == 1 else x_in.stride(1))
                else:
                    x_st, x_sb = B * D, D
                wo = p[pre + "self_attn.output_proj.weight"]
                if cv_nbrs is not None:
                    # the cross-view sub-layer sits between the self-attention residual and the text cross-attention's
                    # LN-mod (the library path computes that LN-mod here too and drops it)
                    fused = self._fused_res(o.view(n * Bs, D), wo, Bs, geo.hw)
                    x, _ = self._proj_res(o.view(n * Bs, D), wo, pre + "self_attn.output_proj", x, x_st, x_sb, g_sa, Bs,
                                          geo, n, lnk, None if fused else sh, None if fused else sc)
                    x, h = self._cross_view(i, x, B, geo, cv_nbrs, mods[i, 1], lnk, sh, sc)
                else:
                    x, h = self._proj_res(o.view(n * Bs, D), wo, pre + "self_attn.output_proj", x, x_st, x_sb, g_sa, Bs,
                                          geo, n, lnk, sh, sc)
            if prefix_only:
                return x, h
            # ---- cross attention (a shared query is read with batch stride 0 against each entry's text K/V)
            xq_scale, xattn_kw = self._attn_mode(self.xattn_bounds[i], hd)  # prescaled q as in self-attention
            hq, wq = _rows(h, n * Bs), p[pre + "cross_attn.q_proj.weight"]
            qc = None
            if self._own(hq, wq):  # the q RMSNorm (+ prescale) in the GEMM's epilogue (cp25_gemm_hnorm, bit-identical)
                qc = N.gemm_hnorm(hq, wq, p[pre + "cross_attn.q_norm.weight"], out_scale=xq_scale)
            if qc is None:
                qc = self._proj(hq, wq, pre + "cross_attn.q_proj")
                N.head_rmsnorm_rope(qc, n_rows=n * Bs, B=Bs, H=H, head_off=0,
                                    weight=p[pre + "cross_attn.q_norm.weight"], out_scale=xq_scale)
            o = torch.empty((n, B, D), dtype=BF16, device=self.device)
            self._cross_attention(qc.view(n, Bs, H, hd).expand(n, B, H, hd), ctx.k[i], ctx.v[i], o.view(n, B, H, hd),
                                  geo, xattn_kw)
            _, _, g_ca = mod(i, 1)
            sh, sc, _ = mod(i, 2)
            x, h = self._proj_res(o.view(n * B, D), p[pre + "cross_attn.output_proj.weight"], pre + "cross_attn.output_proj",
                                  x, Bs * D, 0 if Bs == 1 else D, g_ca, B, geo, n, lnk, sh, sc)
            # ---- MLP
            h1 = _rows(h, n * B)
            w1, w2 = p[pre + "mlp.layer1.weight"], p[pre + "mlp.layer2.weight"]
            _, _, g_ml = mod(i, 2)
            last = i + 1 == cfg.num_blocks
            sh, sc = (None, None) if last else mod(i + 1, 0)[:2]
            if self._own(h1, w1):
                # layer1 + exact-erf GELU in one hand-written MFMA GEMM (the epilogue applies it to the bf16 product, as
                # cp25_gelu would): the [n B, 4 D] hidden makes one HBM trip instead of three
                u = N.gemm_epi(h1, w1, epilogue=N.EPI_GELU)
            else:  # fp8 option: the GELU rides in layer2's row quantisation
                u = self._linear(h1, w1, pre + "mlp.layer1")
            if self._fused_res(u, w2, B, geo.hw):
                x, h = self._proj_res(u, w2, pre + "mlp.layer2", x, B * D, D, g_ml, B, geo, n, lnk, sh, sc,
                                      gelu_in=self.linear_precision == "fp8")
                y, gate_prev = None, None
            else:
                y = self._linear(u, w2, pre + "mlp.layer2", gelu_in=self.linear_precision != "bf16")
                gate_prev = g_ml
                if not last:
                    x_new = torch.empty((n, B, D), dtype=BF16, device=self.device)
                    h = N.ln_mod(x, sh, sc, x_st=B * D, x_sb=D, y=y, gate=gate_prev, x_out=x_new, **lnk)
                    x = x_new
            del u
            if cp is None or cp_size == 1:
                yield i
        # ---- final layer (fp32 autocast): x + g*y -> LN -> modulate -> Linear(D -> 64)
        if not cfg.use_wan_fp32_strategy:
            # FinalLayer without the fp32 autocast (minimal_v4_dit.py:974-995): LayerNorm, * (1 + scale), + shift as
            # bf16 ops (cp25_ln_mod's arithmetic, with the last residual) and a bf16 linear on the own GEMM
            x_new = torch.empty((n, B, D), dtype=BF16, device=self.device) if y is not None else None
            h = N.ln_mod(x, shift_f, scale_f, x_st=B * D, x_sb=D, y=y, gate=gate_prev, x_out=x_new, **common)
            out = N.gemm_epi(h.view(n * B, D), self.w_final_bf16)[:, : self.w_final.shape[0]].float()
            return out.view(n, B, -1)
        xf = N.final_ln_mod(x, shift_f, scale_f, y=y, gate=gate_prev, **common)
        out = N.gemm_f32(xf.view(n * B, D), self.w_final, split_k=False)  # rows independent of the shard size
        return out.view(n, B, -1)

    def _cross_attention(self, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, o: torch.Tensor, geo: Geometry,
                         attn_kw: dict) -> None:
        """Text cross-attention of this shard's queries q/o [n, B, H, hd] against k/v [B, Lc, H, hd].
        Multi-view context holds 512 tokens per view and each view's queries see only their own
        (MultiViewCrossAttention, multiview_dit.py:40-55); a shard may span view boundaries."""
        n = q.shape[0]
        n_ctx = k.shape[1] // 512 if k.shape[1] % 512 == 0 else 1
        if geo.n_views == 1 or n_ctx == 1:
            N.attn_fwd(q.transpose(0, 1), k, v, out=o.transpose(0, 1), **attn_kw)
            return
        if n_ctx != geo.n_views:
            raise ValueError(f"context has {n_ctx} x 512 tokens for {geo.n_views} views")
        for vi in range(geo.n_views):
            a = max(geo.tok0, vi * geo.L_view) - geo.tok0
            b = min(geo.tok0 + n, (vi + 1) * geo.L_view) - geo.tok0
            if a >= b:
                continue
            ks = slice(vi * 512, (vi + 1) * 512)
            N.attn_fwd(q[a:b].transpose(0, 1), k[:, ks], v[:, ks], out=o[a:b].transpose(0, 1), **attn_kw)

    def _kv_gather_buffer(self, shape) -> torch.Tensor:
        """The all-gather's destination for one lane-block's K|V rows (a fresh caching-allocator buffer; the one-GPU
        rank simulation, tools/sim_cp_rank.py --gather none, substitutes a persistent pre-filled one)."""
        return torch.empty(shape, dtype=BF16, device=self.device)

    def _cp_self_attention(self, i: int, h: torch.Tensor, o: torch.Tensor, cos, sin, n: int, B: int, cp,
                           cp_size: int, e0=None, views: Optional[Geometry] = None):
        """Self-attention of a context-parallel token shard (replaces the reference's Ulysses
        all-to-all, a2a_cp.py:160-219, which needs T % cp == 0): the shard's normed + roped K|V rows
        are all-gathered from every rank over RCCL, asynchronously (the other lane computes
        meanwhile); the attention waits for the gather only. Same QKV GEMM and norm as CP = 1.
        views (a frame-sharded cross-view rank's local geometry): per-view self-attention, view v's keys are every
        rank's rows of view v in rank order, i.e. in frame order (copied into one sequence per view)."""
        cfg = self.cfg
        p = self.sd
        pre = f"blocks.{i}."
        D, H, hd = cfg.model_channels, cfg.num_heads, cfg.head_dim
        qkv = self._qkv_k_normed(h, i, n * B, B, cos, sin)  # [n*B, 3D], k normed + roped
        # (q and k|v as two GEMMs, the gather reading the k|v GEMM's output with no export copy, measured 0.25 % slower
        # per CP = 8 rank forward in a same-process A/B: profiles/r5/cp_sim/split_qkv_ab_rejected.log)
        kv = torch.empty((n * B, 2 * D), dtype=BF16, device=self.device)
        N.copy_rows(qkv, 3 * D, kv, 2 * D, n * B, 2 * D, src_offset=D)
        kv_all = self._kv_gather_buffer((cp_size * n * B, 2 * D))
        work = all_gather_into_async(kv_all, kv, cp)  # RCCL over xGMI
        yield i  # the other lane's block runs here (in issue order) while this gather is in flight
        q_scale, attn_kw = self._self_attn_mode(i, hd)
        if self._q_norm_in_attention(attn_kw):
            attn_kw = dict(attn_kw, q_norm=dict(weight=p[pre + "self_attn.q_norm.weight"], cos=cos, sin=sin,
                                                out_scale=q_scale))
        else:
            N.head_rmsnorm_rope(qkv, n_rows=n * B, B=B, H=H, head_off=0, weight=p[pre + "self_attn.q_norm.weight"],
                                cos=cos, sin=sin, out_scale=q_scale)
        w_ev = None
        if self.comm_events is not None:
            w_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            w_ev[0].record()
        work.wait()
        if w_ev is not None:
            w_ev[1].record()
            self.comm_events.append(w_ev)
        if views is not None:
            if self.attention_precision != "bf16":
                raise NotImplementedError("the fp8 attention forms are not built for per-view self-attention")
            if e0 is not None:
                e0.record()
            V, Lv = views.n_views, views.L_view
            q = qkv.view(n, B, 3 * D)[:, :, :D].view(n, B, H, hd).transpose(0, 1)
            ov = o.view(n, B, H, hd).transpose(0, 1)
            kv5 = kv_all.view(cp_size, V, Lv * B, 2 * D)
            qn = attn_kw.get("q_norm")
            for vi in range(V):
                kc, vc = kv_chunk_views(kv5[:, vi].reshape(cp_size * Lv * B, 2 * D), cp_size * Lv, B, H, hd)
                sl = slice(vi * Lv, (vi + 1) * Lv)
                kw = attn_kw if qn is None else dict(attn_kw, q_norm=dict(qn, cos=qn["cos"][sl], sin=qn["sin"][sl]))
                N.attn_fwd(q[:, sl], kc, vc, out=ov[:, sl], **kw)
            return
        kc, vc = kv_chunk_views(kv_all, cp_size * n, B, H, hd)
        attn_kw = self._fp8_qk(qkv[:, :D], kv_all[:, :D], B, H, hd, attn_kw, vc)
        if e0 is not None:
            e0.record()
        q = qkv.view(n, B, 3 * D)[:, :, :D].view(n, B, H, hd).transpose(0, 1)
        # the library's key-range split plan: B = 1 launches at CP = 8 leave a ragged last round
        N.attn_fwd(q, kc, vc, out=o.view(n, B, H, hd).transpose(0, 1), **attn_kw)

    # ---------------------------------------------------------------- reference-compatible forward
    @torch.no_grad()
    def forward(self, x_B_C_T_H_W: torch.Tensor, timesteps_B_T: torch.Tensor, crossattn_emb: torch.Tensor,
                condition_video_input_mask_B_C_T_H_W: Optional[torch.Tensor] = None, fps=None,
                padding_mask: Optional[torch.Tensor] = None, data_type=None, action: Optional[torch.Tensor] = None,
                **kwargs) -> torch.Tensor:
        """MinimalV1LVGDiT.forward signature (minimal_v1_lvg_dit.py:31-62; action nets:
        action_conditioned_minimal_v1_lvg_dit.py:236-249) -> [B, C, T, H, W] fp32."""
        cfg = self.cfg
        B, C, T, Hl, Wl = x_B_C_T_H_W.shape
        Hp, Wp = Hl // cfg.patch_spatial, Wl // cfg.patch_spatial
        geo = Geometry(T=T, Hp=Hp, Wp=Wp, tok0=0, n_tok=T * Hp * Wp, n_views=self.n_views_for(T))
        view_indices = None
        vi_bt = kwargs.get("view_indices_B_T")
        if vi_bt is not None and cfg.n_cameras_emb:  # [B, V*T] -> one index per view (multiview_dit.py:474-478)
            view_indices = vi_bt[0, ::geo.T_view]
        x = x_B_C_T_H_W.to(self.device, BF16)
        if condition_video_input_mask_B_C_T_H_W is None:
            mask = torch.zeros(B, 1, T, Hl, Wl, dtype=BF16, device=self.device)
        else:
            mask = condition_video_input_mask_B_C_T_H_W.to(self.device).to(BF16)
        chans = [x, mask]
        if cfg.concat_padding_mask:
            pm = padding_mask if padding_mask is not None else torch.zeros(B, 1, Hl, Wl)
            pm = F.interpolate(pm.to(self.device).float(), size=(Hl, Wl), mode="nearest").to(BF16)
            chans.append(pm[:, :, None].expand(B, 1, T, Hl, Wl))
        xc = torch.cat(chans, dim=1)
        # b c t (h m) (w n) -> (t h w) b (c m n)
        rows = xc.view(B, xc.shape[1], T, Hp, 2, Wp, 2).permute(2, 3, 5, 0, 1, 4, 6).reshape(geo.L, B, -1)
        ctx = self.prepare_context(crossattn_emb)
        if timesteps_B_T.ndim == 1:
            timesteps_B_T = timesteps_B_T.unsqueeze(1)
        t = self.scale_timesteps(timesteps_B_T)
        if t.shape[1] == 1 and T > 1:
            t = t.expand(B, T).contiguous()
        out = self.forward_tokens(rows.contiguous(), t, ctx, geo, action=action,
                                  view_indices=view_indices)  # [L, B, 64] (p1 p2 C)
        out = out.view(T, Hp, Wp, B, 2, 2, C).permute(3, 6, 0, 1, 4, 2, 5)
        return out.reshape(B, C, T, Hl, Wl).float()

    __call__ = forward
