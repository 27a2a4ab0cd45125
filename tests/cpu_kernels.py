"""Test-only CPU stand-ins for the libcp25 entry points the DiT forward calls (cosmos_predict2._native), so the
CP host path -- dit.forward_tokens driving its two lanes through context_parallel.run_lanes with real
asynchronous gloo all-gathers -- runs on a CPU-only machine. Each function keeps its _native signature and computes
the reference's op sequence with torch CPU ops (the same formulas as oracle/dit.py); none of this is product code
and the product never imports it (the product raises without libcp25.so).

usage: with cpu_kernels.patched(): ...   (monkeypatches cosmos_predict2._native in place)
"""
import contextlib
import math

import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N

BF16 = torch.bfloat16


def _rows_of(t, n, B, tok0, hw):
    """[B', T, D] modulation view -> [n, B, D] rows (frame (tok0 + tok) // hw, batch entry b)."""
    fr = (tok0 + torch.arange(n)) // hw
    return t[:B, fr].transpose(0, 1)


def _view(x, n, B, D, st, sb):
    return torch.as_strided(x, (n, B, D), (st, sb, 1), x.storage_offset())


def ln_mod(x, shift, scale, *, n_tok, B, tok0, hw, x_st, x_sb, y=None, gate=None, x_out=None, h_out=None,
           eps=1e-6, fp8=False):
    if fp8:
        raise NotImplementedError("fp8 LN-mod has no CPU stand-in")
    D = shift.shape[-1]
    xv = _view(x, n_tok, B, D, x_st, x_sb)
    if y is not None:
        xv = xv + _rows_of(gate, n_tok, B, tok0, hw) * y.view(n_tok, B, D)
        if x_out is not None:
            x_out.copy_(xv)
    h = F.layer_norm(xv, (D,), eps=eps) * (1 + _rows_of(scale, n_tok, B, tok0, hw)) + _rows_of(shift, n_tok, B, tok0, hw)
    if h_out is None:
        return h.contiguous()
    h_out.copy_(h)
    return h_out


def final_ln_mod(x, shift, scale, *, n_tok, B, tok0, hw, y=None, gate=None, eps=1e-6):
    D = shift.shape[-1]
    xv = x.view(n_tok, B, D)
    if y is not None:
        xv = xv + _rows_of(gate, n_tok, B, tok0, hw) * y.view(n_tok, B, D)
    return (F.layer_norm(xv.float(), (D,), eps=eps) * (1 + _rows_of(scale, n_tok, B, tok0, hw))
            + _rows_of(shift, n_tok, B, tok0, hw))


def head_rmsnorm_rope(buf, *, n_rows, B, H, head_off, weight, cos=None, sin=None, out2=None, out2_stride=0, eps=1e-6,
                      out_scale=1.0):
    if out2 is not None:
        raise NotImplementedError
    cols = buf[:n_rows, head_off:head_off + H * 128].view(n_rows, H, 128)
    xf = cols.float()
    xn = ((xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)) * weight.float()).to(BF16).float()
    if cos is not None:
        tok = torch.arange(n_rows) // B
        c = torch.cat([cos, cos], -1)[tok][:, None, :]
        s = torch.cat([sin, sin], -1)[tok][:, None, :]
        xn = xn * c + torch.cat([-xn[..., 64:], xn[..., :64]], -1) * s
    cols.copy_((xn * out_scale).to(BF16))


def copy_rows(src, src_stride, dst, dst_stride, n_rows, width, src_offset=0):
    s = torch.as_strided(src, (n_rows, width), (src_stride, 1), src.storage_offset() + src_offset)
    torch.as_strided(dst, (n_rows, width), (dst_stride, 1), dst.storage_offset()).copy_(s)


def attn_fwd(q, k, v, out=None, softmax_scale=None, n_split=None, norm_bounds=None, prescaled=False, fp8_qk=None,
             fp8_v=None, k_norm_slots=None, q_norm=None):
    if fp8_qk is not None or fp8_v is not None:
        raise NotImplementedError
    D = q.shape[-1]
    if q_norm is not None:  # the in-kernel q normalisation: head_rmsnorm_rope's arithmetic on a copy of q
        Bq, Lq, H = q.shape[:3]
        qq = q.transpose(0, 1).contiguous().view(Lq * Bq, H * D)
        head_rmsnorm_rope(qq, n_rows=Lq * Bq, B=Bq, H=H, head_off=0, weight=q_norm["weight"], cos=q_norm.get("cos"),
                          sin=q_norm.get("sin"), eps=q_norm.get("eps", 1e-6), out_scale=q_norm.get("out_scale", 1.0))
        q = qq.view(Lq, Bq, H, D).transpose(0, 1)
    c = math.log(2.0) if prescaled else (D ** -0.5 if softmax_scale is None else softmax_scale)
    s = torch.einsum("blhd,bmhd->bhlm", q.float(), k.float()) * c
    o = torch.einsum("bhlm,bmhd->blhd", torch.softmax(s, -1), v.float()).to(BF16)
    if out is None:
        return o
    out.copy_(o)
    return out


def attn_kernel_name(*a, **kw):
    return "cpu stand-in"


def gemm_epi(a, w, epilogue=N.EPI_NONE, out=None):
    y = F.linear(a, w)
    if epilogue == N.EPI_GELU:
        y = F.gelu(y)
    if out is None:
        return y
    out.copy_(y)
    return out


def gemm_f32(a, w, add=None, act=N.ACT_NONE, out=None, split_k=True):
    y = torch.matmul(a, w.transpose(-1, -2))
    if add is not None:
        y = y + add
    if act == N.ACT_SILU:
        y = F.silu(y)
    if out is None:
        return y
    out.copy_(y)
    return out


def gemm_res(a, w, x, x_st, x_sb, gate, *, B, tok0, hw, out=None):
    M, Nn = a.shape[0], w.shape[0]
    n = M // B
    r = _view(x, n, B, Nn, x_st, x_sb) + _rows_of(gate, n, B, tok0, hw) * F.linear(a, w).view(n, B, Nn)
    if out is None:
        return r.reshape(M, Nn)
    out.view(n, B, Nn).copy_(r)
    return out


def layer_norm(x, weight, bias, eps=1e-6, out=None):
    y = F.layer_norm(x.float(), (x.shape[-1],), weight.float(), bias.float(), eps=eps).to(BF16)
    if out is None:
        return y
    out.copy_(y)
    return out


def gelu_(x):
    x.copy_(F.gelu(x))
    return x


# ---- VAE entry points (the banded decode's host path on the CPU). Computed in float64 and rounded once to bf16, so an
# output pixel does not depend on how much of the image a call covers (a band plus halo rows, or the whole frame).
def conv3d(frames, weight, bias, out, *, Hin, Win, Cin, Cout, Tout, KT, KH, KW, stride_t=1, stride_hw=1,
           pad=(0, 0, 0, 0), upsample=False, out_split=0, residual=None):
    x = torch.stack([f.double() if f is not None else torch.zeros(Hin, Win, Cin, dtype=torch.float64) for f in frames])
    x = x.permute(3, 0, 1, 2)[None]  # [1, C, F, H, W]
    if upsample:
        x = x.repeat_interleave(2, 3).repeat_interleave(2, 4)
    top, left, bottom, right = pad
    x = F.pad(x, (left, right, top, bottom))  # negative pads crop
    w = weight.double().permute(0, 4, 1, 2, 3)  # [Cout, Cin, KT, KH, KW]
    y = F.conv3d(x, w, None if bias is None else bias.double(), stride=(stride_t, stride_hw, stride_hw))[0, :, :Tout]
    y = y.permute(1, 2, 3, 0)  # [Tout, Ho, Wo, Cout]
    if out_split:  # time_conv of upsample3d: channel halves -> frames 2t, 2t + 1
        y = y.reshape(Tout, y.shape[1], y.shape[2], 2, out_split).permute(0, 3, 1, 2, 4).reshape(2 * Tout, y.shape[1],
                                                                                                   y.shape[2], out_split)
    y = y.to(BF16)
    if residual is not None:
        y = (y.double() + residual.double()).to(BF16)
    out.copy_(y)
    return out


def rms_norm_silu(x, gamma, silu=True, out=None):
    xf = x.double()
    y = xf / xf.norm(2, dim=-1, keepdim=True).clamp_min(1e-12) * (x.shape[-1] ** 0.5) * gamma.double()
    if silu:
        y = F.silu(y)
    y = y.to(BF16)
    if out is None:
        return y
    out.copy_(y)
    return out


def gemm_hnorm(a, w, norm_weight, *, out_scale=1.0, eps=1e-6, out=None):
    y = F.linear(a, w)
    head_rmsnorm_rope(y, n_rows=y.shape[0], B=1, H=y.shape[1] // 128, head_off=0, weight=norm_weight, eps=eps,
                      out_scale=out_scale)
    if out is None:
        return y
    out.copy_(y)
    return out


def gemm_qkv(a, w, k_norm_weight, *, k_col0, k_cols, B, cos=None, sin=None, eps=1e-6, out=None):
    y = F.linear(a, w)
    head_rmsnorm_rope(y, n_rows=y.shape[0], B=B, H=k_cols // 128, head_off=k_col0, weight=k_norm_weight, cos=cos,
                      sin=sin, eps=eps)
    if out is None:
        return y
    out.copy_(y)
    return out


def vae_attn(q, k, v, out=None, scale=None):
    sc = q.shape[-1] ** -0.5 if scale is None else scale
    p = torch.softmax(torch.einsum("tld,tmd->tlm", q.double(), k.double()) * sc, -1)
    o = torch.einsum("tlm,tmd->tld", p, v.double()).to(BF16)
    if out is None:
        return o
    out.copy_(o)
    return out


_FUNCS = dict(conv3d=conv3d, rms_norm_silu=rms_norm_silu, vae_attn=vae_attn, ln_mod=ln_mod, final_ln_mod=final_ln_mod, head_rmsnorm_rope=head_rmsnorm_rope, copy_rows=copy_rows,
              attn_fwd=attn_fwd, attn_kernel_name=attn_kernel_name, gemm_epi=gemm_epi, gemm_f32=gemm_f32, gemm_res=gemm_res,
              gemm_hnorm=gemm_hnorm, gemm_qkv=gemm_qkv, gelu_=gelu_, layer_norm=layer_norm)


@contextlib.contextmanager
def patched():
    saved = {k: getattr(N, k) for k in _FUNCS}
    for k, f in _FUNCS.items():
        setattr(N, k, f)
    try:
        yield
    finally:
        for k, f in saved.items():
            setattr(N, k, f)
