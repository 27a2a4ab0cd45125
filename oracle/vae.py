"""Wan2.1 causal video VAE restatement (CPU, NCTHW) — TEST INFRASTRUCTURE (see oracle/__init__.py).

Follows cosmos_predict2/_src/predict2/tokenizers/wan2pt1.py:
  CausalConv3d :44-62 (2 frames of front temporal padding, or the cached frames)
  RMS_norm :65-77, Upsample :80-85, Resample :88-162 (incl. the "Rep" first-chunk rule :117-141 and
  the downsample3d cache :147-161), ResidualBlock :188-222, AttentionBlock :225-261,
  Encoder3d :264-359, Decoder3d :362-458, WanVAE_.encode/decode :504-570 (chunking: first frame
  alone, then temporal_window frames; decode one latent frame at a time), WanVAE scale :726-764,
  Wan2pt1VAEInterface.encode/decode :998-1026 (img/video mean-std identity when load_mean_std=False).
The model runs in bf16 (is_amp=False, wan2pt1.py:790-792): every op rounds to bf16 as torch does.
Convolutions accumulate in fp32 (parity unpinned: cuDNN in the reference).
fp32_truth(): the same restatement over the same bf16 weights with every activation kept in fp32 (no intermediate
bf16 rounding): the exact-math scale both the bf16 reference and the HIP path are measured against.
Device-agnostic torch code: the tests run it on the CPU, and at the 704 x 1280 geometry (minutes on host cores) on the
GPU's own torch ops (MIOpen / hipBLASLt in fp32), never on this repository's kernels.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16
CACHE_T = 2
_ACT = [BF16]  # activation dtype: bf16 = the reference's arithmetic; fp32 inside fp32_truth()


def act_dtype() -> torch.dtype:
    return _ACT[-1]


@contextlib.contextmanager
def fp32_truth():
    _ACT.append(torch.float32)
    try:
        yield
    finally:
        _ACT.pop()

MEAN = [-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
        0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921]
STD = [2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
       3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160]


def _conv3d(x, w, b, pad_hw, cache=None, pt=None):
    """CausalConv3d: 2*padding_t zero frames in front (minus cached frames), symmetric spatial.
    pt defaults to 2 for a temporal kernel of 3 (padding 1) and 0 otherwise."""
    if pt is None:
        pt = 2 if w.shape[2] == 3 else 0
    if cache is not None and pt > 0:
        x = torch.cat([cache.to(x.dtype), x], dim=2)
        pt -= cache.shape[2]
    x = F.pad(x, (pad_hw, pad_hw, pad_hw, pad_hw, pt, 0))
    return F.conv3d(x.float(), w.float(), b.float()).to(x.dtype)


def _conv2d(x, w, b, stride=1, padding=0):
    return F.conv2d(x.float(), w.float(), b.float(), stride=stride, padding=padding).to(x.dtype)


def rms_norm(x, gamma, channel_dim=1):
    n = x.float().norm(2, dim=channel_dim, keepdim=True).to(x.dtype).clamp_min(1e-12)
    y = x / n
    y = y * (x.shape[channel_dim] ** 0.5)
    return y * gamma.to(x.dtype) + 0.0


def silu(x):
    return F.silu(x.float()).to(x.dtype)


class _Cache:
    """feat_cache / feat_idx bookkeeping of the reference (one slot per CausalConv3d)."""

    def __init__(self):
        self.slots = {}
        self.idx = 0

    def reset_idx(self):
        self.idx = 0


def _cached_conv(sd, name, x, cache: _Cache, pad_hw=1):
    """The `cache_x = x[:, :, -2:]; ...; x = conv(x, feat_cache[idx]); feat_cache[idx] = cache_x` idiom."""
    w, b = sd[name + ".weight"], sd[name + ".bias"]
    if cache is None:
        return _conv3d(x, w, b, pad_hw)
    i = cache.idx
    prev = cache.slots.get(i)
    cache_x = x[:, :, -CACHE_T:].clone()
    if cache_x.shape[2] < 2 and prev is not None:
        cache_x = torch.cat([prev[:, :, -1:].to(cache_x.device), cache_x], dim=2)
    out = _conv3d(x, w, b, pad_hw, prev)
    cache.slots[i] = cache_x
    cache.idx += 1
    return out


def res_block(sd, p, x, cache):
    cin = sd[p + ".residual.2.weight"].shape[1]
    cout = sd[p + ".residual.2.weight"].shape[0]
    h = _conv3d(x, sd[p + ".shortcut.weight"], sd[p + ".shortcut.bias"], 0) if cin != cout else x
    y = silu(rms_norm(x, sd[p + ".residual.0.gamma"]))
    y = _cached_conv(sd, p + ".residual.2", y, cache)
    y = silu(rms_norm(y, sd[p + ".residual.3.gamma"]))
    y = _cached_conv(sd, p + ".residual.6", y, cache)
    return y + h


def attn_block(sd, p, x):
    identity = x
    b, c, t, h, w = x.shape
    y = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    y = rms_norm(y, sd[p + ".norm.gamma"])
    qkv = _conv2d(y, sd[p + ".to_qkv.weight"], sd[p + ".to_qkv.bias"])
    qkv = qkv.reshape(b * t, 1, c * 3, -1).permute(0, 1, 3, 2).contiguous()
    q, k, v = qkv.chunk(3, dim=-1)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * (c ** -0.5)
    o = torch.matmul(torch.softmax(s, -1), v.float()).to(x.dtype)
    o = o.squeeze(1).permute(0, 2, 1).reshape(b * t, c, h, w)
    o = _conv2d(o, sd[p + ".proj.weight"], sd[p + ".proj.bias"])
    o = o.reshape(b, t, c, h, w).permute(0, 2, 1, 3, 4)
    return o + identity


def resample(sd, p, mode, x, cache: _Cache):
    b, c, t, h, w = x.shape
    if mode == "upsample3d" and cache is not None:
        i = cache.idx
        prev = cache.slots.get(i)
        if prev is None:
            cache.slots[i] = "Rep"
            cache.idx += 1
        else:
            cache_x = x[:, :, -CACHE_T:].clone()
            if cache_x.shape[2] < 2 and not isinstance(prev, str):
                cache_x = torch.cat([prev[:, :, -1:], cache_x], dim=2)
            if cache_x.shape[2] < 2 and isinstance(prev, str):
                cache_x = torch.cat([torch.zeros_like(cache_x), cache_x], dim=2)
            wt, bt = sd[p + ".time_conv.weight"], sd[p + ".time_conv.bias"]
            x = _conv3d(x, wt, bt, 0, None if isinstance(prev, str) else prev)
            cache.slots[i] = cache_x
            cache.idx += 1
            x = x.reshape(b, 2, c, t, h, w)
            x = torch.stack((x[:, 0], x[:, 1]), 3).reshape(b, c, t * 2, h, w)
    t = x.shape[2]
    y = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    if mode.startswith("upsample"):
        y = F.interpolate(y.float(), scale_factor=2.0, mode="nearest-exact").to(y.dtype)
        y = _conv2d(y, sd[p + ".resample.1.weight"], sd[p + ".resample.1.bias"], padding=1)
    else:
        y = F.pad(y, (0, 1, 0, 1))
        y = _conv2d(y, sd[p + ".resample.1.weight"], sd[p + ".resample.1.bias"], stride=2)
    x = y.reshape(b, t, y.shape[1], y.shape[2], y.shape[3]).permute(0, 2, 1, 3, 4)
    if mode == "downsample3d" and cache is not None:
        i = cache.idx
        prev = cache.slots.get(i)
        if prev is None:
            cache.slots[i] = x.clone()
            cache.idx += 1
        else:
            cache_x = x[:, :, -1:].clone()
            x = _conv3d(torch.cat([prev[:, :, -1:], x], 2), sd[p + ".time_conv.weight"],
                        sd[p + ".time_conv.bias"], 0, pt=0)
            # stride (2,1,1): keep every other output frame
            x = x[:, :, ::2]
            cache.slots[i] = cache_x
            cache.idx += 1
    return x


def encoder_layout(dim=96, dim_mult=(1, 2, 4, 4), nres=2, tdown=(False, True, True)):
    dims = [dim * u for u in (1,) + tuple(dim_mult)]
    layers = []
    for i, (cin, cout) in enumerate(zip(dims[:-1], dims[1:])):
        for _ in range(nres):
            layers.append(("res", cin, cout))
            cin = cout
        if i != len(dim_mult) - 1:
            layers.append(("downsample3d" if tdown[i] else "downsample2d", cout, cout))
    return layers, dims[-1]


def decoder_layout(dim=96, dim_mult=(1, 2, 4, 4), nres=2, tup=(True, True, False)):
    dims = [dim * u for u in (dim_mult[-1],) + tuple(dim_mult[::-1])]
    layers = []
    for i, (cin, cout) in enumerate(zip(dims[:-1], dims[1:])):
        if i in (1, 2, 3):
            cin = cin // 2
        for _ in range(nres + 1):
            layers.append(("res", cin, cout))
            cin = cout
        if i != len(dim_mult) - 1:
            layers.append(("upsample3d" if tup[i] else "upsample2d", cout, cout))
    return layers, dims


def encoder3d(sd, x, cache):
    x = _cached_conv(sd, "encoder.conv1", x, cache)
    layers, _ = encoder_layout()
    for i, (kind, _, _) in enumerate(layers):
        p = f"encoder.downsamples.{i}"
        x = res_block(sd, p, x, cache) if kind == "res" else resample(sd, p, kind, x, cache)
    x = res_block(sd, "encoder.middle.0", x, cache)
    x = attn_block(sd, "encoder.middle.1", x)
    x = res_block(sd, "encoder.middle.2", x, cache)
    x = silu(rms_norm(x, sd["encoder.head.0.gamma"]))
    return _cached_conv(sd, "encoder.head.2", x, cache)


def decoder3d(sd, x, cache):
    x = _cached_conv(sd, "decoder.conv1", x, cache)
    x = res_block(sd, "decoder.middle.0", x, cache)
    x = attn_block(sd, "decoder.middle.1", x)
    x = res_block(sd, "decoder.middle.2", x, cache)
    layers, _ = decoder_layout()
    for i, (kind, _, _) in enumerate(layers):
        p = f"decoder.upsamples.{i}"
        x = res_block(sd, p, x, cache) if kind == "res" else resample(sd, p, kind, x, cache)
    x = silu(rms_norm(x, sd["decoder.head.0.gamma"]))
    return _cached_conv(sd, "decoder.head.2", x, cache)


def _scale(device="cpu"):
    # the buffers are bf16 in the reference (the whole VAE is cast to bf16); the truth keeps those values
    mean = torch.tensor(MEAN, dtype=BF16).to(device=device, dtype=act_dtype())
    std = torch.tensor(STD, dtype=BF16).to(device=device, dtype=act_dtype())
    return mean, 1.0 / std


def encode(sd, video: torch.Tensor, temporal_window: int = 16) -> torch.Tensor:
    """video [B, 3, T, H, W] in [-1, 1] -> latent mu [B, 16, 1 + (T-1)//4, H/8, W/8] (bf16)."""
    x = video.to(BF16).to(act_dtype())  # the same (bf16-valued) input pixels in both modes
    t = x.shape[2]
    cache = _Cache()
    outs = []
    n_iter = 1 + (t - 1) // temporal_window
    for i in range(n_iter):
        cache.reset_idx()
        if i == 0:
            chunk = x[:, :, :1]
        else:
            chunk = x[:, :, 1 + temporal_window * (i - 1): 1 + temporal_window * i]
        outs.append(encoder3d(sd, chunk, cache))
    if (t - 1) % temporal_window:
        cache.reset_idx()
        outs.append(encoder3d(sd, x[:, :, 1 + temporal_window * (n_iter - 1):], cache))
    out = torch.cat(outs, 2)
    mu = _conv3d(out, sd["conv1.weight"], sd["conv1.bias"], 0).chunk(2, dim=1)[0]
    mean, inv_std = _scale(mu.device)
    return (mu - mean.view(1, 16, 1, 1, 1)) * inv_std.view(1, 16, 1, 1, 1)


def decode(sd, z: torch.Tensor, progress=None) -> torch.Tensor:
    """latent [B, 16, T, h, w] -> video [B, 3, 1 + 4 (T-1), 8h, 8w] (bf16, ~[-1, 1]). progress(i): called after each
    latent frame (long runs report liveness)."""
    mean, inv_std = _scale(z.device)
    z = z.to(act_dtype())
    z = z / inv_std.view(1, 16, 1, 1, 1) + mean.view(1, 16, 1, 1, 1)
    x = _conv3d(z, sd["conv2.weight"], sd["conv2.bias"], 0)
    cache = _Cache()
    outs = []
    for i in range(z.shape[2]):
        cache.reset_idx()
        outs.append(decoder3d(sd, x[:, :, i: i + 1], cache))
        if progress is not None:
            progress(i)
    return torch.cat(outs, 2)
