"""Wan2.1 causal video VAE (the Cosmos-Predict2.5 tokenizer) for MI355X.

Same weights (tokenizer.pth keys encoder.* / conv1.* / conv2.* / decoder.*), same chunking and
causal feature-cache semantics as the reference (cosmos_predict2/_src/predict2/tokenizers/wan2pt1.py:
Encoder3d :264-359, Decoder3d :362-458, WanVAE_.encode/decode :504-570, Wan2pt1VAEInterface :961-1060),
re-laid-out for the GPU:
* activations are channels-last clips [T][H][W][C] bf16, so every convolution is an implicit GEMM
  over (kt, kh, kw, cin) with contiguous channel vectors (cp25_conv3d, bf16 MFMA);
* the causal padding / feat_cache of every CausalConv3d is a table of frame pointers handed to the
  kernel (zero frames are NULL), never a concatenated copy;
* nearest-2x upsampling is fused into the conv's input gather, the upsample3d frame interleave into
  its epilogue, bias + residual adds into the conv epilogue; RMS_norm + SiLU is one HIP kernel.
The single-head AttentionBlock core (C = 384 at h/8 x w/8) is the flash kernel cp25_vae_attn reading q / k / v
straight out of the to_qkv output (no score matrix in HBM); its 1x1 projections and norm are the HIP conv /
norm kernels.

Context parallel decode (set_context_parallel_group): the reference replicates the VAE on every rank;
here each rank decodes a band of h/N latent rows (8h/N output rows) of every frame. A 3x3 conv needs
one input row beyond its band on each side: `_halo` fetches the neighbours' edge rows (RCCL
all-gather of the bands' first/last rows; zero rows at the image edge = the conv's zero padding)
and the conv runs unpadded in h over the haloed band (causal caches keep the haloed frames, so the
cached frames carry their halos too); the nearest-2x upsample conv reads the haloed low-res band with
pads (-1, -1), the (3,1,1) time_conv and 1x1 convs need no halo, RMS_norm is per pixel, and the
middle AttentionBlock gathers K/V of the whole frame. Bands are gathered into the full video at the
end. Every output pixel is computed from the same inputs in the same order as the unbanded decode.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from . import _native as N
from . import context_parallel as cpx

BF16 = torch.bfloat16
CACHE_T = 2
MAX_FRAMES = 24  # frame-table size of cp25_conv3d

_MEAN = [-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
         0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921]
_STD = [2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
        3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160]


# ----------------------------------------------------------------------------- layout
def encoder_layers(dim=96, dim_mult=(1, 2, 4, 4), nres=2, tdown=(False, True, True)):
    dims = [dim * u for u in (1,) + tuple(dim_mult)]
    out = []
    for i, (cin, cout) in enumerate(zip(dims[:-1], dims[1:])):
        for _ in range(nres):
            out.append(("res", cin, cout))
            cin = cout
        if i != len(dim_mult) - 1:
            out.append(("downsample3d" if tdown[i] else "downsample2d", cout, cout))
    return out


def decoder_layers(dim=96, dim_mult=(1, 2, 4, 4), nres=2, tup=(True, True, False)):
    dims = [dim * u for u in (dim_mult[-1],) + tuple(dim_mult[::-1])]
    out = []
    for i, (cin, cout) in enumerate(zip(dims[:-1], dims[1:])):
        if i in (1, 2, 3):
            cin //= 2
        for _ in range(nres + 1):
            out.append(("res", cin, cout))
            cin = cout
        if i != len(dim_mult) - 1:
            out.append(("upsample3d" if tup[i] else "upsample2d", cout, cout))
    return out


def vae_state_dict_shapes(dim=96, z_dim=16) -> Dict[str, tuple]:
    s: Dict[str, tuple] = {}

    def conv(name, cout, cin, k):
        s[name + ".weight"] = (cout, cin) + k
        s[name + ".bias"] = (cout,)

    def res(p, cin, cout):
        s[p + ".residual.0.gamma"] = (cin, 1, 1, 1)
        conv(p + ".residual.2", cout, cin, (3, 3, 3))
        s[p + ".residual.3.gamma"] = (cout, 1, 1, 1)
        conv(p + ".residual.6", cout, cout, (3, 3, 3))
        if cin != cout:
            conv(p + ".shortcut", cout, cin, (1, 1, 1))

    def attn(p, c):
        s[p + ".norm.gamma"] = (c, 1, 1)
        conv(p + ".to_qkv", 3 * c, c, (1, 1))
        conv(p + ".proj", c, c, (1, 1))

    def resample(p, kind, c):
        if kind.startswith("upsample"):
            conv(p + ".resample.1", c // 2, c, (3, 3))
            if kind == "upsample3d":
                conv(p + ".time_conv", 2 * c, c, (3, 1, 1))
        else:
            conv(p + ".resample.1", c, c, (3, 3))
            if kind == "downsample3d":
                conv(p + ".time_conv", c, c, (3, 1, 1))

    conv("encoder.conv1", dim, 3, (3, 3, 3))
    for i, (k, ci, co) in enumerate(encoder_layers(dim)):
        (res if k == "res" else (lambda p, a, b, kk=k: resample(p, kk, a)))(f"encoder.downsamples.{i}", ci, co)
    top = 4 * dim
    res("encoder.middle.0", top, top)
    attn("encoder.middle.1", top)
    res("encoder.middle.2", top, top)
    s["encoder.head.0.gamma"] = (top, 1, 1, 1)
    conv("encoder.head.2", 2 * z_dim, top, (3, 3, 3))
    conv("conv1", 2 * z_dim, 2 * z_dim, (1, 1, 1))
    conv("conv2", z_dim, z_dim, (1, 1, 1))
    conv("decoder.conv1", top, z_dim, (3, 3, 3))
    res("decoder.middle.0", top, top)
    attn("decoder.middle.1", top)
    res("decoder.middle.2", top, top)
    for i, (k, ci, co) in enumerate(decoder_layers(dim)):
        (res if k == "res" else (lambda p, a, b, kk=k: resample(p, kk, a)))(f"decoder.upsamples.{i}", ci, co)
    s["decoder.head.0.gamma"] = (dim, 1, 1, 1)
    conv("decoder.head.2", 3, dim, (3, 3, 3))
    return s


def init_vae_state_dict(seed: int = 0, device="cpu") -> Dict[str, torch.Tensor]:
    """Seeded synthetic weights (kaiming-uniform convs as nn.Conv default; gammas ~1)."""
    g = torch.Generator(device=device).manual_seed(seed)
    out = {}
    for k, shp in vae_state_dict_shapes().items():
        if k.endswith("gamma"):
            out[k] = (1 + 0.1 * torch.randn(shp, generator=g, device=device)).to(BF16)
        elif k.endswith("bias"):
            out[k] = (0.02 * torch.randn(shp, generator=g, device=device)).to(BF16)
        else:
            fan_in = math.prod(shp[1:])
            bound = 1.0 / math.sqrt(fan_in)
            out[k] = ((torch.rand(shp, generator=g, device=device) * 2 - 1) * bound * math.sqrt(3)).to(BF16)
    return out


# ----------------------------------------------------------------------------- conv helpers
class _Conv:
    """One convolution with device weights repacked [Cout][KT][KH][KW][Cin_pad]."""

    def __init__(self, w: torch.Tensor, b: Optional[torch.Tensor], device, out_rows: Optional[int] = None):
        if w.dim() == 4:
            w = w.unsqueeze(2)  # Conv2d -> KT = 1
        if out_rows is not None:
            w = w[:out_rows]
            b = b[:out_rows] if b is not None else None
        cout, cin, kt, kh, kw = w.shape
        cin_p = ((cin + 15) // 16) * 16
        wp = torch.zeros((cout, kt, kh, kw, cin_p), dtype=BF16, device=device)
        wp[..., :cin] = w.to(device=device, dtype=BF16).permute(0, 2, 3, 4, 1)
        self.w = wp.contiguous()
        self.b = b.to(device=device, dtype=BF16).contiguous() if b is not None else None
        self.cout, self.cin, self.cin_p, self.kt, self.kh, self.kw = cout, cin, cin_p, kt, kh, kw

    def __call__(self, frames: List[Optional[torch.Tensor]], Tout: int, H: int, W: int, *, stride_t=1, stride_hw=1,
                 pad=(0, 0, 0, 0), upsample=False, out_split=0, residual=None) -> torch.Tensor:
        dev = self.w.device
        Hu, Wu = (2 * H, 2 * W) if upsample else (H, W)
        Ho = (Hu + pad[0] + pad[2] - self.kh) // stride_hw + 1
        Wo = (Wu + pad[1] + pad[3] - self.kw) // stride_hw + 1
        if out_split:
            out = torch.empty((2 * Tout, Ho, Wo, out_split), dtype=BF16, device=dev)
        else:
            out = torch.empty((Tout, Ho, Wo, self.cout), dtype=BF16, device=dev)
        # the kernel takes at most MAX_FRAMES input frames per launch: chunk the output frames
        per = max(1, (MAX_FRAMES - self.kt) // stride_t + 1)
        f = 2 if out_split else 1
        for t0 in range(0, Tout, per):
            t1 = min(Tout, t0 + per)
            fr = frames[t0 * stride_t: (t1 - 1) * stride_t + self.kt]
            N.conv3d(fr, self.w, self.b, out[f * t0: f * t1], Hin=H, Win=W, Cin=self.cin_p, Cout=self.cout,
                     Tout=t1 - t0, KT=self.kt, KH=self.kh, KW=self.kw, stride_t=stride_t, stride_hw=stride_hw,
                     pad=pad, upsample=upsample, out_split=out_split,
                     residual=None if residual is None else residual[f * t0: f * t1])
        return out


def _frames(x: torch.Tensor) -> List[torch.Tensor]:
    return [x[i] for i in range(x.shape[0])]


class _FeatCache:
    def __init__(self):
        self.slots: Dict[int, object] = {}
        self.idx = 0


class WanVAE:
    """Encoder/decoder over channels-last clips; B = 1 (the sampler's batch)."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], device="cuda", dim=96, z_dim=16,
                 temporal_window: int = 16):
        self.device = torch.device(device)
        self.dim, self.z_dim, self.temporal_window = dim, z_dim, temporal_window
        sd = {k: v for k, v in state_dict.items()}
        self.convs: Dict[str, _Conv] = {}
        self.gammas: Dict[str, torch.Tensor] = {}
        for k, v in sd.items():
            if k.endswith(".weight"):
                name = k[: -len(".weight")]
                if name == "conv1":  # only mu = the first z_dim output channels is ever used
                    self.convs[name] = _Conv(v, sd.get(name + ".bias"), self.device, out_rows=z_dim)
                else:
                    self.convs[name] = _Conv(v, sd.get(name + ".bias"), self.device)
            elif k.endswith(".gamma"):
                self.gammas[k[: -len(".gamma")]] = v.to(self.device, BF16).reshape(-1).contiguous()
        mean = torch.tensor(_MEAN, dtype=BF16, device=self.device)
        std = torch.tensor(_STD, dtype=BF16, device=self.device)
        self.mean, self.inv_std = mean, 1.0 / std
        self.cp_group = None  # decode shards latent rows over this group (see module docstring)
        self._band = None  # (group, rank, world) while a banded decode runs

    # ---------------------------------------------------------------- context-parallel bands
    def _halo(self, x: torch.Tensor) -> torch.Tensor:
        """[T, R, W, C] band -> [T, R + 2, W, C] with the neighbouring bands' edge rows (zeros at the
        image's top and bottom edge)."""
        group, r, n = self._band
        T, R, W, C = x.shape
        xh = torch.empty((T, R + 2, W, C), dtype=x.dtype, device=x.device)
        xh[:, 1:R + 1] = x
        edge = torch.stack([x[:, 0], x[:, R - 1]], 0)  # [2, T, W, C]
        allv = torch.empty((n,) + tuple(edge.shape), dtype=x.dtype, device=x.device)
        cpx.all_gather_into(allv, edge, group)
        if r > 0:
            xh[:, 0] = allv[r - 1, 1]
        else:
            xh[:, 0].zero_()
        if r < n - 1:
            xh[:, R + 1] = allv[r + 1, 0]
        else:
            xh[:, R + 1].zero_()
        return xh

    # ---------------------------------------------------------------- building blocks
    def _causal(self, name, x, cache: Optional[_FeatCache], H, W):
        """CausalConv3d 3x3x3 (pad 1) with the feat_cache rule (wan2pt1.py:206-219)."""
        conv = self.convs[name]
        pad = (1, 1, 1, 1)
        if self._band is not None:
            x = self._halo(x)
            H, pad = H + 2, (0, 1, 0, 1)
        T = x.shape[0]
        prev = None
        if cache is not None:
            i = cache.idx
            prev = cache.slots.get(i)
            cache_x = x[-CACHE_T:].clone()
            if cache_x.shape[0] < 2 and prev is not None:
                cache_x = torch.cat([prev[-1:], cache_x], 0)
            cache.slots[i] = cache_x
            cache.idx += 1
        pre: List[Optional[torch.Tensor]] = [None, None]
        if prev is not None:
            pre = [None] * (2 - prev.shape[0]) + _frames(prev)
        return conv(pre + _frames(x), T, H, W, pad=pad)

    def _res(self, p, x, cache, H, W, cin, cout):
        if cin != cout:
            h = self.convs[p + ".shortcut"](_frames(x), x.shape[0], H, W)
        else:
            h = x
        y = N.rms_norm_silu(x, self.gammas[p + ".residual.0"], silu=True)
        y = self._causal_res(p + ".residual.2", y, cache, H, W)
        y = N.rms_norm_silu(y, self.gammas[p + ".residual.3"], silu=True)
        return self._causal_res(p + ".residual.6", y, cache, H, W, residual=h)

    def _causal_res(self, name, x, cache, H, W, residual=None):
        conv = self.convs[name]
        pad = (1, 1, 1, 1)
        if self._band is not None:
            x = self._halo(x)
            H, pad = H + 2, (0, 1, 0, 1)
        T = x.shape[0]
        i = cache.idx
        prev = cache.slots.get(i)
        cache_x = x[-CACHE_T:].clone()
        if cache_x.shape[0] < 2 and prev is not None:
            cache_x = torch.cat([prev[-1:], cache_x], 0)
        cache.slots[i] = cache_x
        cache.idx += 1
        pre: List[Optional[torch.Tensor]] = [None, None] if prev is None else [None] * (2 - prev.shape[0]) + _frames(prev)
        return conv(pre + _frames(x), T, H, W, pad=pad, residual=residual)

    def _attn(self, p, x, H, W):
        C = x.shape[-1]
        T = x.shape[0]
        y = N.rms_norm_silu(x, self.gammas[p + ".norm"], silu=False)
        qkv = self.convs[p + ".to_qkv"](_frames(y), T, H, W)  # [T, H, W, 3C]
        qkv = qkv.view(T, H * W, 3 * C)
        q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]
        if self._band is not None:  # K/V of the whole frame: every band's rows, in row order
            group, _, n = self._band
            kv = qkv[:, :, C:].contiguous()
            kv_all = torch.empty((n,) + tuple(kv.shape), dtype=BF16, device=self.device)
            cpx.all_gather_into(kv_all, kv, group)
            kv_all = kv_all.permute(1, 0, 2, 3).reshape(T, n * H * W, 2 * C)  # [T, all rows, 2C]
            k, v = kv_all[:, :, :C], kv_all[:, :, C:]
        # F.scaled_dot_product_attention(q, k, v) on bf16, one head (wan2pt1.py:251-254): the flash kernel
        # cp25_vae_attn (fp32 scores, bf16 P), no score matrix in HBM
        o = N.vae_attn(q, k, v)
        o = o.view(T, H, W, C)
        return self.convs[p + ".proj"](_frames(o), T, H, W, residual=x)

    def _resample(self, p, kind, x, cache, H, W):
        T = x.shape[0]
        if kind == "upsample3d" and cache is not None:
            i = cache.idx
            prev = cache.slots.get(i)
            if prev is None:
                cache.slots[i] = "Rep"
                cache.idx += 1
            else:
                cache_x = x[-CACHE_T:].clone()
                if cache_x.shape[0] < 2 and not isinstance(prev, str):
                    cache_x = torch.cat([prev[-1:], cache_x], 0)
                if cache_x.shape[0] < 2 and isinstance(prev, str):
                    cache_x = torch.cat([torch.zeros_like(cache_x), cache_x], 0)
                pre = [None, None] if isinstance(prev, str) else [None] * (2 - prev.shape[0]) + _frames(prev)
                x = self.convs[p + ".time_conv"](pre + _frames(x), T, H, W, out_split=x.shape[-1])
                cache.slots[i] = cache_x
                cache.idx += 1
        T = x.shape[0]
        conv = self.convs[p + ".resample.1"]
        if kind.startswith("upsample") and self._band is not None:
            # haloed low-res band; in upsampled coordinates the output rows start one row in: pads -1
            xh = self._halo(x)
            y = conv(_frames(xh), T, H + 2, W, pad=(-1, 1, -1, 1), upsample=True)
            H, W = 2 * H, 2 * W
        elif kind.startswith("upsample"):
            y = conv(_frames(x), T, H, W, pad=(1, 1, 1, 1), upsample=True)
            H, W = 2 * H, 2 * W
        else:
            y = conv(_frames(x), T, H, W, stride_hw=2, pad=(0, 0, 1, 1))
            H, W = H // 2, W // 2
        if kind == "downsample3d" and cache is not None:
            i = cache.idx
            prev = cache.slots.get(i)
            if prev is None:
                cache.slots[i] = y.clone()
                cache.idx += 1
            else:
                cache_x = y[-1:].clone()
                fr = [prev[-1]] + _frames(y)
                tout = (len(fr) - 3) // 2 + 1
                y = self.convs[p + ".time_conv"](fr, tout, H, W, stride_t=2)
                cache.slots[i] = cache_x
                cache.idx += 1
        return y, H, W

    # ---------------------------------------------------------------- encoder / decoder
    def _encoder(self, x, cache, H, W):
        x = self._causal("encoder.conv1", x, cache, H, W)
        for i, (kind, ci, co) in enumerate(encoder_layers(self.dim)):
            p = f"encoder.downsamples.{i}"
            if kind == "res":
                x = self._res(p, x, cache, H, W, ci, co)
            else:
                x, H, W = self._resample(p, kind, x, cache, H, W)
        top = 4 * self.dim
        x = self._res("encoder.middle.0", x, cache, H, W, top, top)
        x = self._attn("encoder.middle.1", x, H, W)
        x = self._res("encoder.middle.2", x, cache, H, W, top, top)
        x = N.rms_norm_silu(x, self.gammas["encoder.head.0"], silu=True)
        return self._causal("encoder.head.2", x, cache, H, W), H, W

    def _decoder(self, x, cache, H, W):
        x = self._causal("decoder.conv1", x, cache, H, W)
        top = 4 * self.dim
        x = self._res("decoder.middle.0", x, cache, H, W, top, top)
        x = self._attn("decoder.middle.1", x, H, W)
        x = self._res("decoder.middle.2", x, cache, H, W, top, top)
        for i, (kind, ci, co) in enumerate(decoder_layers(self.dim)):
            p = f"decoder.upsamples.{i}"
            if kind == "res":
                x = self._res(p, x, cache, H, W, ci, co)
            else:
                x, H, W = self._resample(p, kind, x, cache, H, W)
        x = N.rms_norm_silu(x, self.gammas["decoder.head.0"], silu=True)
        return self._causal("decoder.head.2", x, cache, H, W), H, W

    @torch.no_grad()
    def encode(self, video: torch.Tensor) -> torch.Tensor:
        """video [1, 3, T, H, W] (bf16 in [-1, 1]) -> mu [1, 16, 1 + (T-1)//4, H/8, W/8] bf16."""
        assert video.shape[0] == 1, "batch 1"
        _, C, T, H, W = video.shape
        x = torch.zeros((T, H, W, 16), dtype=BF16, device=self.device)  # channels padded 3 -> 16
        x[..., :C] = video[0].to(self.device, BF16).permute(1, 2, 3, 0)
        cache = _FeatCache()
        tw = self.temporal_window
        chunks = [x[:1]]
        n_iter = 1 + (T - 1) // tw
        for i in range(1, n_iter):
            chunks.append(x[1 + tw * (i - 1): 1 + tw * i])
        if (T - 1) % tw:
            chunks.append(x[1 + tw * (n_iter - 1):])
        outs = []
        for ch in chunks:
            cache.idx = 0
            o, h, w = self._encoder(ch.contiguous(), cache, H, W)
            outs.append(o)
        out = torch.cat(outs, 0)
        mu = self.convs["conv1"](_frames(out), out.shape[0], h, w)  # [Tl, h, w, 16]
        mu = (mu - self.mean) * self.inv_std
        return mu.permute(3, 0, 1, 2).unsqueeze(0).contiguous()

    @torch.no_grad()
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        """latent [1, 16, T, h, w] -> video [1, 3, 1 + 4 (T-1), 8h, 8w] bf16."""
        assert z.shape[0] == 1, "batch 1"
        _, C, T, h, w = z.shape
        zl = z[0].to(self.device, BF16).permute(1, 2, 3, 0).contiguous()  # [T, h, w, 16]
        zl = zl / self.inv_std + self.mean
        group = self.cp_group
        r, n = cpx.cp_rank_world(group)
        if n > 1 and h % n == 0:
            self._band = (group, r, n)
            zl = zl[:, r * (h // n):(r + 1) * (h // n)]
            h = h // n
        try:
            x = self.convs["conv2"](_frames(zl.contiguous()), T, h, w)
            cache = _FeatCache()
            outs = []
            for i in range(T):
                cache.idx = 0
                o, H, W = self._decoder(x[i: i + 1].contiguous(), cache, h, w)
                outs.append(o)
            video = torch.cat(outs, 0)  # [Tp, H, W, 3] (this rank's band of H rows when banded)
            if self._band is not None:
                allv = torch.empty((n,) + tuple(video.shape), dtype=video.dtype, device=video.device)
                cpx.all_gather_into(allv, video, group)
                video = allv.permute(1, 0, 2, 3, 4).reshape(video.shape[0], n * video.shape[1], *video.shape[2:])
        finally:
            self._band = None
        return video.permute(3, 0, 1, 2).unsqueeze(0).contiguous()


class Wan2pt1VAEInterface:
    """VideoTokenizerInterface of the reference (tokenizers/interface.py:25-98, wan2pt1.py:961-1060)."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], device="cuda", temporal_window: int = 16,
                 chunk_duration: int = 81):
        self.model = WanVAE(state_dict, device=device, temporal_window=temporal_window)
        self.chunk_duration = chunk_duration

    def set_context_parallel_group(self, group) -> None:
        """Decode shards latent rows over `group` (WanVAE module docstring); encode stays replicated."""
        self.model.cp_group = group

    def encode(self, state: torch.Tensor) -> torch.Tensor:
        in_dtype = state.dtype
        return self.model.encode(state).to(in_dtype)

    def decode(self, latent: torch.Tensor) -> torch.Tensor:
        in_dtype = latent.dtype
        return self.model.decode(latent).to(in_dtype)

    def get_latent_num_frames(self, num_pixel_frames: int) -> int:
        return 1 + (num_pixel_frames - 1) // 4

    def get_pixel_num_frames(self, num_latent_frames: int) -> int:
        return (num_latent_frames - 1) * 4 + 1

    @property
    def spatial_compression_factor(self) -> int:
        return 8

    @property
    def temporal_compression_factor(self) -> int:
        return 4

    @property
    def latent_ch(self) -> int:
        return 16

    @property
    def pixel_chunk_duration(self) -> int:
        return self.chunk_duration

    @property
    def latent_chunk_duration(self) -> int:
        return self.get_latent_num_frames(self.chunk_duration)

    @property
    def spatial_resolution(self) -> int:
        return 512

    @property
    def name(self) -> str:
        return "wan2pt1_tokenizer"
