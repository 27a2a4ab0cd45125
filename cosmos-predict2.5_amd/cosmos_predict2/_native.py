"""ctypes binding of libcp25.so (the C ABI declared in include/cp25.h).

This module is the only place the Python host code touches native kernels. It fails loudly: if the
library is missing or a device tensor is not on a ROCm GPU, it raises instead of falling back to a
PyTorch/CPU implementation (there is no fallback path in the product).
"""

from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import torch

_DEFAULT_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libcp25.so")
_LIB_PATH = _DEFAULT_LIB_PATH
_lib: Optional[ctypes.CDLL] = None

c_int64_p = ctypes.POINTER(ctypes.c_int64)


class UniPCParams(ctypes.Structure):
    """Mirror of `cp25_unipc_params` (include/cp25.h)."""

    _fields_ = [
        ("sigma", ctypes.c_float),
        ("use_corr", ctypes.c_int),
        ("order_c", ctypes.c_int),
        ("c_a", ctypes.c_float),
        ("c_b", ctypes.c_float),
        ("c_c", ctypes.c_float),
        ("c_inv_rk", ctypes.c_float),
        ("c_rho0", ctypes.c_float),
        ("c_rho_last", ctypes.c_float),
        ("order_p", ctypes.c_int),
        ("p_a", ctypes.c_float),
        ("p_b", ctypes.c_float),
        ("p_c", ctypes.c_float),
        ("p_inv_rk", ctypes.c_float),
        ("p_rho0", ctypes.c_float),
    ]


class CP25Tensor(ctypes.Structure):
    """Mirror of `cp25_tensor` (include/cp25.h): device pointer, CP25_DT_* dtype, rank, sizes, strides (elements)."""

    _fields_ = [
        ("data", ctypes.c_void_p),
        ("dtype", ctypes.c_int32),
        ("ndim", ctypes.c_int32),
        ("shape", ctypes.c_int64 * 6),
        ("strides", ctypes.c_int64 * 6),
    ]


DT_BF16, DT_F32, DT_F8E4M3, DT_U8 = 1, 2, 3, 4
_DTYPES = {torch.bfloat16: DT_BF16, torch.float32: DT_F32, torch.float8_e4m3fn: DT_F8E4M3, torch.uint8: DT_U8}

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_F = ctypes.c_float
_T = ctypes.POINTER(CP25Tensor)

# symbol -> argtypes (restype int, except the *_workspace_bytes queries)
SIGNATURES = {
    "cp25_attn_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, c_int64_p, _F, _P],
    "cp25_attn_fwd_split": [_P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, c_int64_p, _F, _I,
                            _P, ctypes.c_size_t, _P],
    "cp25_attn_fwd_bounded": [_P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, c_int64_p, _F, _F,
                              _F, _I, _P, ctypes.c_size_t, _P],
    "cp25_attn_fwd_prescaled_kslots": [_P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, c_int64_p,
                                       _F, _F, _P, _I, _I, _P, ctypes.c_size_t, _P],
    "cp25_attn_fwd_prescaled": [_P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, c_int64_p, _F,
                                _F, _I, _P, ctypes.c_size_t, _P],
    "cp25_attn_fwd_prescaled_fp8qk": [_P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, c_int64_p, _F,
                                _F, _I, _P, ctypes.c_size_t, _P],
    "cp25_cast_fp8_e4m3": [_P, _I64, _P, _I64, _I64, _I64, _F, _P],
    "cp25_attn_fwd_prescaled_fp8": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, _F, _F, _I,
                                    _P, ctypes.c_size_t, _P],
    "cp25_v_fp8t_bytes": [_I, _I, _I],
    "cp25_cast_v_fp8t": [_P, c_int64_p, _I, _I, _I, _I, _P, _P, _P],
    "cp25_attn_fwd_prescaled_qnorm": [_P, _P, _P, _P, _I, _I, _I, _I, _I, c_int64_p, c_int64_p, c_int64_p, c_int64_p, _F,
                                      _F, _P, _I, _P, _P, _P, _F, _F, _I, _P, ctypes.c_size_t, _P],
    "cp25_attn_workspace_bytes": [_I, _I, _I, _I],
    "cp25_attn_tail_workspace_bytes": [_I, _I, _I, _I],
    "cp25_attn_kernel": [_I, _F, _F, _F, _I, _I],
    "cp25_attn_plan": [_I, _I, _I, _I, _I],
    "cp25_ln_mod": [_P, _I64, _I64, _P, _P, _P, _P, _I64, _I64, _P, _P, _I64, _I, _I, _I64, _I64, _F, _P],
    "cp25_ln_mod_fp8": [_P, _I64, _I64, _P, _P, _P, _P, _I64, _I64, _P, _P, _P, _I64, _I, _I, _I64, _I64, _F, _P],
    "cp25_final_ln_mod": [_P, _P, _P, _I64, _I64, _P, _P, _I64, _I64, _P, _I64, _I, _I, _I64, _I64, _F, _P],
    "cp25_layer_norm": [_P, _I64, _P, _P, _P, _I64, _I64, _I, _F, _P],
    "cp25_head_rmsnorm_rope": [_P, _I64, _I64, _I, _I, _I, _P, _P, _P, _P, _I64, _F, _P],
    "cp25_head_rmsnorm_rope_scaled": [_P, _I64, _I64, _I, _I, _I, _P, _P, _P, _P, _I64, _F, _F, _P],
    "cp25_head_rmsnorm_rope_nmax": [_P, _I64, _I64, _I, _I, _I, _P, _P, _P, _P, _I64, _F, _F, _P, _P],
    "cp25_copy_rows": [_P, _I64, _P, _I64, _I64, _I64, _P],
    "cp25_gelu": [_P, _I64, _P],
    "cp25_gemm_epi": [_P, _I64, _P, _I64, _P, _I64, _I, _I, _I, _I, _P],
    "cp25_gemm_f32": [_P, _I64, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _I64, _I64, _I, _I, _I, _I, _I, _P, _I64,
                      _P],
    "cp25_gemm_f32_workspace_floats": [_I, _I, _I, _I],
    "cp25_gemm_hnorm": [_P, _I64, _P, _I64, _P, _I64, _I, _I, _I, _P, _F, _F, _P],
    "cp25_gemm_qkv": [_P, _I64, _P, _I64, _P, _I64, _I, _I, _I, _I, _I, _P, _P, _P, _I, _F, _P],
    "cp25_gemm_res": [_P, _I64, _P, _I64, _P, _I64, _I, _I, _I, _P, _I64, _I64, _P, _I64, _I64, _I, _I64, _I64, _P],
    "cp25_gemm_fp8": [_P, _I64, _P, _P, _I64, _P, _P, _I64, _I, _I, _I, _P],
    "cp25_gemm_fp8_res": [_P, _I64, _P, _P, _I64, _P, _P, _I64, _I, _I, _I, _P, _I64, _I64, _P, _I64, _I64, _I, _I64,
                          _I64, _P],
    "cp25_quant_fp8_rows": [_P, _P, _P, _I64, _I64, _P],
    "cp25_gelu_quant_fp8": [_P, _P, _P, _I64, _I64, _P],
    "cp25_patchify": [_P, _P, _P, _P, _P, _I64, _I64, _I64, _P],
    "cp25_patchify_ld": [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _P],
    "cp25_cfg_velocity": [_P, _I, _P, _P, _P, _F, _I, _P, _I64, _I64, _I64, _P],
    "cp25_unipc_step": [_P, _P, _P, _P, _P, _I64, ctypes.POINTER(UniPCParams), _P],
    "cp25_conv3d": [ctypes.POINTER(ctypes.c_void_p), _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I,
                    _I, _I, _I, _I, _I, _I, _P],
    "cp25_rms_norm_silu": [_P, _P, _P, _I64, _I, _I, _P],
    "cp25_conv3d_select": [_I],
    "cp25_attn_cross_select": [_I],
    "cp25_softmax_rows": [_P, _I64, _I, _I64, _F, _P, _I64, _P],
    "cp25_vae_attn": [_P, _I64, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _I64, _I64, _I, _I, _I, _I, _F, _P, _I64,
                      _P],
    "cp25_vae_attn_workspace_bytes": [_I, _I, _I, _I],
    "cp25_attn_fwd_t": [_T, _T, _T, _T, _F, _P, ctypes.c_size_t, _P],
    "cp25_gemm_epi_t": [_T, _T, _T, _I, _P],
    "cp25_conv3d_t": [_T, _I, _T, _T, _T, _I, _I, _I, _I, _I, _I, _P],
}


def library_path() -> str:
    return _LIB_PATH


def load_library() -> ctypes.CDLL:
    """Load libcp25.so (import torch first so the HIP runtime torch ships is the one bound)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise RuntimeError(
            f"libcp25.so not found at {_LIB_PATH}: build it with `make -C cosmos-predict2.5_amd/csrc` "
            "(or __graft_entry__.build()). There is no non-native fallback."
        )
    lib = ctypes.CDLL(_LIB_PATH)
    lab = os.path.abspath(_LIB_PATH) != os.path.abspath(_DEFAULT_LIB_PATH)  # an A/B build (tools/lab): may predate symbols
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if argtypes is None or lab:
                continue
            raise RuntimeError(f"libcp25.so does not export {name}")
        if argtypes is not None:
            fn.argtypes = argtypes
        fn.restype = {"cp25_attn_workspace_bytes": ctypes.c_size_t, "cp25_attn_tail_workspace_bytes": ctypes.c_size_t, "cp25_v_fp8t_bytes": ctypes.c_int64,
                      "cp25_gemm_f32_workspace_floats": ctypes.c_int64,
                      "cp25_attn_kernel": ctypes.c_char_p,
                      "cp25_vae_attn_workspace_bytes": ctypes.c_int64}.get(name, ctypes.c_int)
    _lib = lib
    return lib


_ERRORS = {-22: "invalid shape/stride/pointer", -95: "unsupported dtype/size", -5: "kernel launch failed"}


def _check(name: str, rc: int) -> None:
    if rc != 0:
        msg = f"{name} failed with code {rc} ({_ERRORS.get(rc, 'unknown')})"
        if rc == -5:
            raise RuntimeError(msg)
        raise ValueError(msg)


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("cp25 kernels need device (HBM) tensors; got a CPU tensor")
    return t.data_ptr()


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def tensor_desc(t: Optional[torch.Tensor]) -> Optional[CP25Tensor]:
    """A cp25_tensor for a device tensor (data pointer, dtype, sizes, strides); None for None."""
    if t is None:
        return None
    if t.dim() > 6:
        raise ValueError(f"cp25_tensor holds at most 6 dimensions, got {t.dim()}")
    if t.dtype not in _DTYPES:
        raise ValueError(f"no cp25 dtype for {t.dtype}")
    d = CP25Tensor()
    d.data = _ptr(t)
    d.dtype = _DTYPES[t.dtype]
    d.ndim = t.dim()
    for i in range(t.dim()):
        d.shape[i] = t.shape[i]
        d.strides[i] = t.stride(i)
    return d


def _ref(d: Optional[CP25Tensor]):
    return None if d is None else ctypes.byref(d)


def attn_fwd_t(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, o: torch.Tensor, softmax_scale: float,
               workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """cp25_attn_fwd_t: the descriptor form of the attention (q / o [B, Lq, H, D], k / v [B, Lk, H, D] bf16); the
    library checks dtypes and strides (ValueError on a mismatch)."""
    lib = load_library()
    ws = 0 if workspace is None else workspace.numel() * workspace.element_size()
    _check("cp25_attn_fwd_t", lib.cp25_attn_fwd_t(*(_ref(tensor_desc(t)) for t in (q, k, v, o)), float(softmax_scale),
                                                  _ptr(workspace), ws, _stream(q.device)))
    return o


def gemm_epi_t(a: torch.Tensor, w: torch.Tensor, c: torch.Tensor, epilogue: int = 0) -> torch.Tensor:
    """cp25_gemm_epi_t: c [M, N] = epi(a [M, K] w [N, K]^T) over descriptors (EPI_NONE / EPI_GELU)."""
    lib = load_library()
    _check("cp25_gemm_epi_t", lib.cp25_gemm_epi_t(_ref(tensor_desc(a)), _ref(tensor_desc(w)), _ref(tensor_desc(c)),
                                                  int(epilogue), _stream(a.device)))
    return c


def conv3d_t(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], out: torch.Tensor, *,
             pad_front: int = 0, stride_t: int = 1, stride_hw: int = 1, pad: tuple = (0, 0, 0, 0)) -> torch.Tensor:
    """cp25_conv3d_t: x [T, H, W, C] channels-last frames after pad_front zero frames, weight [Cout, KT, KH, KW, Cin],
    bias [Cout] or None, out [Tout, Ho, Wo, Cout]; pad = (top, left, bottom, right)."""
    lib = load_library()
    _check("cp25_conv3d_t", lib.cp25_conv3d_t(_ref(tensor_desc(x)), int(pad_front), _ref(tensor_desc(weight)),
                                              _ref(tensor_desc(bias)), _ref(tensor_desc(out)), stride_t, stride_hw,
                                              pad[0], pad[1], pad[2], pad[3], _stream(x.device)))
    return out


def _i64x3(vals) -> ctypes.Array:
    arr = (ctypes.c_int64 * 3)(*[int(v) for v in vals])
    return arr


# ----------------------------------------------------------------------------- attention
# Key-range split override, resolved once at import from CP25_ATTN_SPLIT (e.g. "1": never split, for bitwise
# CP = N vs CP = 1 checks; unset: the library's plan); set_attn_split() changes it in-process.
_ATTN_SPLIT: Optional[int] = int(os.environ["CP25_ATTN_SPLIT"]) if os.environ.get("CP25_ATTN_SPLIT") else None


def set_attn_split(n: Optional[int]) -> Optional[int]:
    """Force every attn_fwd call without an explicit n_split to use at most n key-range splits (None: the library's
    plan). Returns the previous setting."""
    global _ATTN_SPLIT
    prev, _ATTN_SPLIT = _ATTN_SPLIT, (None if n is None else int(n))
    return prev


def attn_plan(B: int, H: int, Lq: int, Lk: int, D: int = 128) -> int:
    """Key-range split the library picks for this shape (cp25_attn_plan)."""
    n = load_library().cp25_attn_plan(B, H, Lq, Lk, D)
    _check("cp25_attn_plan", min(n, 0))
    return n


def attn_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: Optional[torch.Tensor] = None,
             softmax_scale: Optional[float] = None, n_split: Optional[int] = None,
             norm_bounds: Optional[Tuple[float, float]] = None, prescaled: bool = False,
             fp8_qk: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
             fp8_v: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
             k_norm_slots: Optional[torch.Tensor] = None, q_norm: Optional[dict] = None) -> torch.Tensor:
    """softmax(q k^T * scale) v for q [B, Lq, H, 128], k/v [B, Lk, H, 128] (bf16, any strides with
    a contiguous head dim). Returns [B, Lq, H, 128] bf16. n_split: key-range split (None = the
    library's plan for this shape; the fp32 partials live in a caching-allocator workspace).
    norm_bounds: (max |q|, max |k|) upper bounds over all rows: where max|q| max|k| (in log2 units) <= 98 the
    rows use a fixed softmax shift, else (or None) an online row max (cp25_attn_fwd_bounded; any data).
    prescaled=True: q rows already carry scale * log2(e) (head_rmsnorm_rope(out_scale=...)); norm_bounds (of the
    scaled q and of k) optional as above (cp25_attn_fwd_prescaled; softmax_scale unused).
    fp8_qk=(q8, k8): with prescaled, Q K^T runs on the e4m3 copies (uint8 views shaped like q / k, from
    cast_fp8(q * 2^s), cast_fp8(k * 2^-s); cp25_attn_fwd_prescaled_fp8qk; needs bounds with product <= 60); q / k
    are then only shape references. fp8_v=(v8t, v_amax) (with fp8_qk; from cast_v_fp8t(v)): P.V on e5m2 P and
    e4m3 V too (cp25_attn_fwd_prescaled_fp8; needs 1.13 x the bound product <= 30); v is then only a shape
    reference. k_norm_slots (with prescaled, bf16): the float32 [64, 32] slots head_rmsnorm_rope(norm_max=...) filled
    for k, a data-tight key bound (cp25_attn_fwd_prescaled_kslots: blocks whose bound allows it run the fixed-shift
    loop even when norm_bounds do not).
    q_norm=dict(weight=w [128] bf16, cos=None|[Lq, 64] fp32, sin=..., eps=1e-6, out_scale=c) (with prescaled, bf16
    attention): q holds the raw projection and the kernel applies head_rmsnorm_rope(weight, cos, sin, out_scale)'s
    arithmetic to its Q fragments as they load, bit for bit (cp25_attn_fwd_prescaled_qnorm): the separate q RMSNorm
    pass over HBM is gone. cos / sin rows are indexed by the query row (token) of q."""
    lib = load_library()
    if q.dtype != torch.bfloat16 or k.dtype != torch.bfloat16 or v.dtype != torch.bfloat16:
        raise ValueError("attn_fwd expects bf16 q/k/v (attention() recasts to bf16 first)")
    B, Lq, H, D = q.shape
    Bk, Lk, Hk, Dk = k.shape
    if (Bk, Hk, Dk) != (B, H, D) or tuple(v.shape) != tuple(k.shape):
        raise ValueError(f"shape mismatch q{tuple(q.shape)} k{tuple(k.shape)} v{tuple(v.shape)}")
    for t in (q, k, v):
        if t.stride(3) != 1:
            raise ValueError("head dim must be contiguous")
    if out is None:
        out = torch.empty((B, Lq, H, D), dtype=torch.bfloat16, device=q.device)
    scale = float(D) ** -0.5 if softmax_scale is None else float(softmax_scale)
    planned = n_split is None and not _ATTN_SPLIT
    if n_split is None:
        n_split = min(_ATTN_SPLIT, (Lk + 63) // 64) if _ATTN_SPLIT else attn_plan(B, H, Lq, Lk, D)
    ws_bytes = lib.cp25_attn_workspace_bytes(B, H, Lq, n_split)
    if planned and n_split == 1 and fp8_qk is None and k_norm_slots is None:
        # the library's plan may run the last partial round of workgroups as a tail split (a forced split, e.g. the
        # bit-exact CP tests' CP25_ATTN_SPLIT=1, runs the launch whole)
        ws_bytes = lib.cp25_attn_tail_workspace_bytes(B, H, Lq, Lk)
    ws = torch.empty(((ws_bytes + 15) // 16 * 4,), dtype=torch.float32, device=q.device) if ws_bytes else None
    qb, kb = (0.0, 0.0) if norm_bounds is None else (float(norm_bounds[0]), float(norm_bounds[1]))
    if not (qb >= 0.0 and kb >= 0.0):
        raise ValueError(f"norm_bounds must be >= 0, got {norm_bounds}")
    strides = [_i64x3((t.stride(0), t.stride(1), t.stride(2))) for t in (q, k, v, out)]
    if prescaled:
        if fp8_qk is not None:
            if q_norm is not None:
                raise ValueError("q_norm: the fp8 forms read e4m3 copies of the normalised q")
            if qb * kb > 60.0 or qb <= 0.0 or kb <= 0.0:
                raise ValueError(f"fp8 Q K^T needs norm bounds with product <= 60, got {norm_bounds}")
            q8, k8 = fp8_qk
            if q8.dtype != torch.uint8 or k8.dtype != torch.uint8 or q8.shape != q.shape or k8.shape != k.shape:
                raise ValueError("fp8_qk: uint8 (e4m3 bit pattern) views shaped like q and k expected")
            if q8.stride(3) != 1 or k8.stride(3) != 1:
                raise ValueError("fp8_qk: head dim must be contiguous")
            strides[0] = _i64x3((q8.stride(0), q8.stride(1), q8.stride(2)))
            strides[1] = _i64x3((k8.stride(0), k8.stride(1), k8.stride(2)))
            if fp8_v is not None:
                if 1.13 * qb * kb > 30.0:
                    raise ValueError(f"fp8 P.V needs 1.13 x the norm-bound product <= 30, got {norm_bounds}")
                v8t, amax = fp8_v
                if v8t.dtype != torch.uint8 or v8t.numel() != lib.cp25_v_fp8t_bytes(B, H, Lk) or \
                        amax.dtype != torch.float32 or amax.numel() < B * H:
                    raise ValueError("fp8_v: (v8t uint8 of cp25_v_fp8t_bytes, v_amax float32 [B*H]) expected")
                rc = lib.cp25_attn_fwd_prescaled_fp8(_ptr(q8), _ptr(k8), _ptr(v8t), _ptr(amax), _ptr(out), B, H, Lq, Lk,
                                                     D, strides[0], strides[1], strides[3], qb, kb, int(n_split),
                                                     _ptr(ws), ws_bytes, _stream(q.device))
                _check("cp25_attn_fwd_prescaled_fp8", rc)
                return out
            rc = lib.cp25_attn_fwd_prescaled_fp8qk(_ptr(q8), _ptr(k8), _ptr(v), _ptr(out), B, H, Lq, Lk, D, *strides,
                                                   qb, kb, int(n_split), _ptr(ws), ws_bytes, _stream(q.device))
            _check("cp25_attn_fwd_prescaled_fp8qk", rc)
            return out
        if k_norm_slots is not None:
            if k_norm_slots.dtype != torch.float32 or k_norm_slots.numel() != 2048 or not k_norm_slots.is_contiguous():
                raise ValueError("k_norm_slots: a contiguous float32 [64, 32] slot buffer expected")
        if q_norm is not None:
            w, cos, sin = q_norm["weight"], q_norm.get("cos"), q_norm.get("sin")
            if w.dtype != torch.bfloat16 or w.numel() != D or not w.is_contiguous() or w.device != q.device:
                raise ValueError("q_norm: weight must be a contiguous bf16 [128] device tensor")
            if (cos is None) != (sin is None):
                raise ValueError("q_norm: cos and sin go together")
            if cos is not None:
                for t in (cos, sin):
                    if t.dtype != torch.float32 or not t.is_contiguous() or t.dim() != 2 or t.shape[1] != 64 or \
                            t.shape[0] < Lq or t.device != q.device:
                        raise ValueError(f"q_norm: cos/sin must be contiguous float32 [>= {Lq}, 64] device tables")
            rc = lib.cp25_attn_fwd_prescaled_qnorm(
                _ptr(q), _ptr(k), _ptr(v), _ptr(out), B, H, Lq, Lk, D, *strides, qb, kb, _ptr(k_norm_slots),
                64 if k_norm_slots is not None else 0, _ptr(w), _ptr(cos), _ptr(sin), float(q_norm.get("eps", 1e-6)),
                float(q_norm.get("out_scale", 1.0)), int(n_split), _ptr(ws), ws_bytes, _stream(q.device))
            _check("cp25_attn_fwd_prescaled_qnorm", rc)
            return out
        if k_norm_slots is not None:
            rc = lib.cp25_attn_fwd_prescaled_kslots(_ptr(q), _ptr(k), _ptr(v), _ptr(out), B, H, Lq, Lk, D, *strides, qb,
                                                    kb, _ptr(k_norm_slots), 64, int(n_split), _ptr(ws), ws_bytes,
                                                    _stream(q.device))
            _check("cp25_attn_fwd_prescaled_kslots", rc)
            return out
        rc = lib.cp25_attn_fwd_prescaled(_ptr(q), _ptr(k), _ptr(v), _ptr(out), B, H, Lq, Lk, D, *strides, qb, kb,
                                         int(n_split), _ptr(ws), ws_bytes, _stream(q.device))
        _check("cp25_attn_fwd_prescaled", rc)
        return out
    if q_norm is not None:
        raise ValueError("q_norm needs prescaled=True (the DiT's attention form)")
    rc = lib.cp25_attn_fwd_bounded(
        _ptr(q), _ptr(k), _ptr(v), _ptr(out), B, H, Lq, Lk, D,
        _i64x3((q.stride(0), q.stride(1), q.stride(2))),
        _i64x3((k.stride(0), k.stride(1), k.stride(2))),
        _i64x3((v.stride(0), v.stride(1), v.stride(2))),
        _i64x3((out.stride(0), out.stride(1), out.stride(2))),
        scale, qb, kb, int(n_split), _ptr(ws), ws_bytes, _stream(q.device),
    )
    _check("cp25_attn_fwd_bounded", rc)
    return out


def attn_cross_select(form: int) -> int:
    """cp25_attn_cross_select: the kernel form of short-key (text cross-attention) launches, 1 = persistent (default),
    0 = one workgroup per query block (A/B and tests; bit-identical). Returns the previous form."""
    rc = load_library().cp25_attn_cross_select(int(form))
    _check("cp25_attn_cross_select", min(rc, 0))
    return rc


def attn_self_select(form: int) -> int:
    """Lab builds only (tools/lab/w64/build_lab.sh, loaded through _LIB_PATH): cp25_attn_self_select, the kernel form
    of prescaled bf16 self-attention launches, 0 = attn_fwd_m16 (the product kernel), 1 = attn_fwd_w64 in the zero- and
    fixed-shift modes, 2 = attn_fwd_w64 in every mode (bit-identical). Returns the previous form."""
    lib = load_library()
    fn = getattr(lib, "cp25_attn_self_select", None)
    if fn is None:
        raise RuntimeError("cp25_attn_self_select: not in this libcp25.so (attn_fwd_w64 is a lab build, "
                           "tools/lab/w64/build_lab.sh)")
    fn.argtypes = [ctypes.c_int]
    fn.restype = ctypes.c_int
    rc = fn(int(form))
    _check("cp25_attn_self_select", min(rc, 0))
    return rc


def attn_kernel_name(Lk: int, softmax_scale: Optional[float] = None, norm_bounds=None, prescaled: bool = False,
                     fp8: int = 0) -> str:
    """The kernel form attn_fwd launches for these arguments (cp25_attn_kernel), e.g.
    'attn_fwd_m16<self, prescaled, online max>'; prescaled = 2: the k_norm_slots form."""
    qb, kb = (0.0, 0.0) if norm_bounds is None else (float(norm_bounds[0]), float(norm_bounds[1]))
    sc = 128 ** -0.5 if softmax_scale is None else float(softmax_scale)
    return load_library().cp25_attn_kernel(int(Lk), sc, qb, kb, int(prescaled), int(fp8)).decode()


def cast_v_fp8t(v: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(v8t, v_amax) for attn_fwd(fp8_v=...): v bf16 [B, L, H, 128] (any strides, contiguous head dim) ->
    the e4m3 V^T tile layout and the per-(b, h) max |v| (cp25_cast_v_fp8t)."""
    lib = load_library()
    if v.dtype != torch.bfloat16 or v.dim() != 4 or v.stride(3) != 1:
        raise ValueError("cast_v_fp8t expects bf16 [B, L, H, 128] with a contiguous head dim")
    B, L, H, D = v.shape
    n = lib.cp25_v_fp8t_bytes(B, H, L)
    _check("cp25_v_fp8t_bytes", min(n, 0))
    v8t = torch.empty((n,), dtype=torch.uint8, device=v.device)
    amax = torch.empty((B * H,), dtype=torch.float32, device=v.device)
    rc = lib.cp25_cast_v_fp8t(_ptr(v), _i64x3((v.stride(0), v.stride(1), v.stride(2))), B, H, L, D, _ptr(v8t),
                              _ptr(amax), _stream(v.device))
    _check("cp25_cast_v_fp8t", rc)
    return v8t, amax


def cast_fp8(src: torch.Tensor, scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """e4m3(bf16 src * scale) as uint8 bit patterns, row by row over the last dim (cp25_cast_fp8_e4m3); src is a
    2-D bf16 view with unit inner stride (e.g. the q or k columns of the fused qkv buffer)."""
    lib = load_library()
    if src.dtype != torch.bfloat16 or src.dim() != 2 or src.stride(1) != 1:
        raise ValueError("cast_fp8 expects a 2-D bf16 view with a contiguous last dim")
    n, w = src.shape
    if out is None:
        out = torch.empty((n, w), dtype=torch.uint8, device=src.device)
    if out.dtype != torch.uint8 or out.shape != src.shape or out.stride(1) != 1:
        raise ValueError("cast_fp8: out must be a uint8 tensor shaped like src")
    rc = lib.cp25_cast_fp8_e4m3(_ptr(src), src.stride(0), _ptr(out), out.stride(0), n, w, float(scale),
                                _stream(src.device))
    _check("cp25_cast_fp8_e4m3", rc)
    return out


# ----------------------------------------------------------------------------- DiT elementwise
def _check_frames(mod: torch.Tensor, *, n_tok: int, B: int, tok0: int, hw: int) -> None:
    """The kernels index modulation rows by frame (tok // hw) and batch: both must be in range."""
    if mod.dim() != 3 or mod.shape[0] < B or hw <= 0 or tok0 < 0 or n_tok < 0:
        raise ValueError(f"modulation {tuple(mod.shape)} does not cover B={B}")
    if n_tok and (tok0 + n_tok - 1) // hw >= mod.shape[1]:
        raise ValueError(f"tokens [{tok0}, {tok0 + n_tok}) reach frame {(tok0 + n_tok - 1) // hw}, "
                         f"but the modulation has {mod.shape[1]} frames")


def _check_mask(frame_mask: torch.Tensor, *, n_tok: int, tok0: int, hw: int) -> None:
    if hw <= 0 or tok0 < 0 or (n_tok and (tok0 + n_tok - 1) // hw >= frame_mask.numel()):
        raise ValueError(f"tokens [{tok0}, {tok0 + n_tok}) with hw={hw} exceed the {frame_mask.numel()}-frame mask")


def ln_mod(x: torch.Tensor, shift: torch.Tensor, scale: torch.Tensor, *, n_tok: int, B: int, tok0: int, hw: int,
           x_st: int, x_sb: int, y: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None,
           x_out: Optional[torch.Tensor] = None, h_out: Optional[torch.Tensor] = None,
           eps: float = 1e-6, fp8: bool = False):
    """h = LN(x [+ gate*y]) * (1 + scale) + shift over token-major [n_tok, B, D] bf16 rows.
    shift/scale/gate are bf16 views [B, T, D] (strides (sb, st, 1), shared by all three).
    fp8=True returns h as the row-scaled fp8 GEMM operand (q [n_tok*B, D] float8_e4m3fn, scale
    [n_tok*B, 1] fp32) instead (cp25_ln_mod_fp8)."""
    lib = load_library()
    D = shift.shape[-1]
    _check_frames(shift, n_tok=n_tok, B=B, tok0=tok0, hw=hw)
    if shift.stride() != scale.stride() or (gate is not None and gate.stride() != shift.stride()):
        raise ValueError("shift/scale/gate must share strides")
    if fp8:
        q = torch.empty((n_tok * B, D), dtype=torch.float8_e4m3fn, device=x.device)
        s = torch.empty((n_tok * B, 1), dtype=torch.float32, device=x.device)
        rc = lib.cp25_ln_mod_fp8(
            _ptr(x), x_st, x_sb, _ptr(y), _ptr(gate), _ptr(shift), _ptr(scale), shift.stride(0), shift.stride(1),
            _ptr(x_out), _ptr(q), _ptr(s), n_tok, B, D, tok0, hw, eps, _stream(x.device),
        )
        _check("cp25_ln_mod_fp8", rc)
        return q, s
    if h_out is None:
        h_out = torch.empty((n_tok, B, D), dtype=torch.bfloat16, device=x.device)
    if shift.stride() != scale.stride() or (gate is not None and gate.stride() != shift.stride()):
        raise ValueError("shift/scale/gate must share strides")
    rc = lib.cp25_ln_mod(
        _ptr(x), x_st, x_sb, _ptr(y), _ptr(gate), _ptr(shift), _ptr(scale), shift.stride(0), shift.stride(1),
        _ptr(x_out), _ptr(h_out), n_tok, B, D, tok0, hw, eps, _stream(x.device),
    )
    _check("cp25_ln_mod", rc)
    return h_out


def final_ln_mod(x: torch.Tensor, shift: torch.Tensor, scale: torch.Tensor, *, n_tok: int, B: int, tok0: int, hw: int,
                 y: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None,
                 eps: float = 1e-6) -> torch.Tensor:
    lib = load_library()
    D = shift.shape[-1]
    _check_frames(shift, n_tok=n_tok, B=B, tok0=tok0, hw=hw)
    if gate is not None:
        _check_frames(gate, n_tok=n_tok, B=B, tok0=tok0, hw=hw)
    out = torch.empty((n_tok, B, D), dtype=torch.float32, device=x.device)
    gsb, gst = (gate.stride(0), gate.stride(1)) if gate is not None else (0, 0)
    if shift.stride() != scale.stride():
        raise ValueError("shift/scale must share strides")
    rc = lib.cp25_final_ln_mod(
        _ptr(x), _ptr(y), _ptr(gate), gsb, gst, _ptr(shift), _ptr(scale), shift.stride(0), shift.stride(1),
        _ptr(out), n_tok, B, D, tok0, hw, eps, _stream(x.device),
    )
    _check("cp25_final_ln_mod", rc)
    return out


def head_rmsnorm_rope(buf: torch.Tensor, *, n_rows: int, B: int, H: int, head_off: int, weight: torch.Tensor,
                      cos: Optional[torch.Tensor] = None, sin: Optional[torch.Tensor] = None,
                      out2: Optional[torch.Tensor] = None, out2_stride: int = 0, eps: float = 1e-6,
                      out_scale: float = 1.0, norm_max: Optional[torch.Tensor] = None) -> None:
    """norm_max: float32 [64, 32] slots (zeroed by the caller; slot i = norm_max[i, 0]) that receive the max |row| of the
    result by atomic max (cp25_head_rmsnorm_rope_nmax): the data-tight key bound attn_fwd(k_norm_slots=...) reads."""
    lib = load_library()
    if norm_max is not None and (norm_max.dtype != torch.float32 or norm_max.numel() != 2048 or not norm_max.is_contiguous()):
        raise ValueError("norm_max: a contiguous float32 [64, 32] slot buffer expected")
    rc = lib.cp25_head_rmsnorm_rope_nmax(
        _ptr(buf), buf.stride(-2) if buf.dim() >= 2 else buf.shape[-1], n_rows, B, H, head_off, _ptr(weight),
        _ptr(cos), _ptr(sin), _ptr(out2), out2_stride, eps, out_scale, _ptr(norm_max), _stream(buf.device),
    )
    _check("cp25_head_rmsnorm_rope", rc)


def copy_rows(src: torch.Tensor, src_stride: int, dst: torch.Tensor, dst_stride: int, n_rows: int, width: int,
              src_offset: int = 0) -> None:
    lib = load_library()
    rc = lib.cp25_copy_rows(_ptr(src) + 2 * src_offset, src_stride, _ptr(dst), dst_stride, n_rows, width,
                            _stream(src.device))
    _check("cp25_copy_rows", rc)


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-6,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Affine LayerNorm over the last dim of bf16 rows x [M, D] (row stride x.stride(0)) -> out [M, D] bf16
    (cp25_layer_norm: fp32 statistics and affine, one rounding)."""
    lib = load_library()
    if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16 or bias.dtype != torch.bfloat16:
        raise ValueError("layer_norm expects bf16 rows, weight and bias")
    if x.dim() != 2 or x.stride(1) != 1 or not weight.is_contiguous() or not bias.is_contiguous():
        raise ValueError("layer_norm: x [M, D] with contiguous rows, contiguous weight / bias")
    M, D = x.shape
    if weight.numel() != D or bias.numel() != D:
        raise ValueError(f"layer_norm weight / bias must have {D} elements")
    if out is None:
        out = torch.empty((M, D), dtype=torch.bfloat16, device=x.device)
    _check("cp25_layer_norm", lib.cp25_layer_norm(_ptr(x), x.stride(0), _ptr(weight), _ptr(bias), _ptr(out),
                                                  out.stride(0), M, D, float(eps), _stream(x.device)))
    return out


def gelu_(x: torch.Tensor) -> torch.Tensor:
    lib = load_library()
    if not x.is_contiguous() or x.dtype != torch.bfloat16:
        raise ValueError("gelu_ expects a contiguous bf16 tensor")
    _check("cp25_gelu", lib.cp25_gelu(_ptr(x), x.numel(), _stream(x.device)))
    return x


EPI_NONE, EPI_GELU, EPI_RES, EPI_HNORM, EPI_QKV = 0, 1, 2, 3, 4


def gemm_supported(N: int, K: int) -> bool:
    """Shapes cp25_gemm_epi is built for (N multiple of 256, K of 64); the sampler raises ValueError for others."""
    return N % 256 == 0 and K % 64 == 0


def gemm_res_supported(N: int, K: int, B: int, hw: int) -> bool:
    """Shapes and row groupings cp25_gemm_res is built for: gemm_supported, and B entries per token dividing the 16
    rows a lane group's gate lookup spans with at least 16 / B tokens per frame (gemm.hip, gemm_launch)."""
    return gemm_supported(N, K) and B > 0 and 16 % B == 0 and hw >= 16 // B


def gemm_epi(a: torch.Tensor, w: torch.Tensor, epilogue: int = EPI_NONE, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[M, N] = epi(a[M, K] w[N, K]^T) in bf16 (cp25_gemm_epi); EPI_GELU applies the exact-erf GELU to the
    bf16 product (GPT2FeedForward layer1 + activation)."""
    lib = load_library()
    if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise ValueError("gemm_epi expects bf16 operands")
    if a.dim() != 2 or w.dim() != 2 or a.shape[1] != w.shape[1] or a.stride(1) != 1 or w.stride(1) != 1:
        raise ValueError(f"gemm_epi shapes a{tuple(a.shape)} w{tuple(w.shape)}: need [M, K] x [N, K], K contiguous")
    M, K = a.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if tuple(out.shape) != (M, N) or out.stride(1) != 1:
        raise ValueError(f"gemm_epi out {tuple(out.shape)} != ({M}, {N})")
    rc = lib.cp25_gemm_epi(_ptr(a), a.stride(0), _ptr(w), w.stride(0), _ptr(out), out.stride(0), M, N, K, int(epilogue),
                           _stream(a.device))
    _check("cp25_gemm_epi", rc)
    return out


ACT_NONE, ACT_SILU = 0, 1


def gemm_f32(a: torch.Tensor, w: torch.Tensor, add: Optional[torch.Tensor] = None, act: int = ACT_NONE,
             out: Optional[torch.Tensor] = None, split_k: bool = True) -> torch.Tensor:
    """out = act(a w^T + add) in fp32 (cp25_gemm_f32): the fp32 conditioning linears (t-embedding, AdaLN-LoRA, final
    layer). a [M, K] with w [N, K], or batched a [nb, M, K] with w [nb, N, K] (a's entries may be strided views, e.g.
    column blocks of one wider matrix). add: broadcastable to the output ([N] bias, [M, N] or [nb, M, N]; strides
    taken as given, stride-0 dimensions broadcast). K % 32 == 0. split_k=False: no K split whatever the shape, so
    every output row's sum is independent of M (token rows of a context-parallel shard)."""
    lib = load_library()
    if a.dtype != torch.float32 or w.dtype != torch.float32:
        raise ValueError("gemm_f32 expects fp32 operands")
    if a.dim() != w.dim() or a.dim() not in (2, 3) or a.shape[-1] != w.shape[-1] or a.stride(-1) != 1 \
            or w.stride(-1) != 1 or (a.dim() == 3 and a.shape[0] != w.shape[0]):
        raise ValueError(f"gemm_f32 shapes a{tuple(a.shape)} w{tuple(w.shape)}: need [(nb,) M, K] x [(nb,) N, K]")
    a3 = a if a.dim() == 3 else a.unsqueeze(0)
    w3 = w if w.dim() == 3 else w.unsqueeze(0)
    nb, M, K = a3.shape
    N = w3.shape[1]
    if out is None:
        out = torch.empty((nb, M, N), dtype=torch.float32, device=a.device)
        if a.dim() == 2:
            out = out[0]
    o3 = out if out.dim() == 3 else out.unsqueeze(0)
    if tuple(o3.shape) != (nb, M, N) or o3.stride(2) != 1 or out.dtype != torch.float32:
        raise ValueError(f"gemm_f32 out {tuple(out.shape)} != ({nb}, {M}, {N}) fp32")
    r, ldr, sr = None, 0, 0
    if add is not None:
        if add.dtype != torch.float32:
            raise ValueError("gemm_f32 addend must be fp32")
        r3 = add.expand(nb, M, N)
        if r3.stride(2) != 1:
            raise ValueError("gemm_f32 addend must be contiguous along N")
        r, ldr, sr = r3, r3.stride(1), r3.stride(0)
    nws = lib.cp25_gemm_f32_workspace_floats(M, N, K, nb) if split_k and K % 32 == 0 else 0
    ws = torch.empty(nws, dtype=torch.float32, device=a.device) if nws else None
    rc = lib.cp25_gemm_f32(_ptr(a3), a3.stride(1), a3.stride(0), _ptr(w3), w3.stride(1), w3.stride(0), _ptr(r), ldr, sr,
                           _ptr(o3), o3.stride(1), o3.stride(0), M, N, K, nb, int(act), _ptr(ws), nws,
                           _stream(a.device))
    _check("cp25_gemm_f32", rc)
    return out


def gemm_hnorm(a: torch.Tensor, w: torch.Tensor, norm_weight: torch.Tensor, *, out_scale: float = 1.0,
               eps: float = 1e-6, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """out[M, N] = per-128-column-head RMSNorm(bf16(a w^T)) * norm_weight * out_scale (cp25_gemm_hnorm), bit-identical
    to gemm_epi followed by head_rmsnorm_rope(out_scale=...) without RoPE (the cross-attention q projection + q_norm).
    None when the kernel is not built for the shape (K / 64 odd): the caller runs the two ops."""
    lib = load_library()
    if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or norm_weight.dtype != torch.bfloat16:
        raise ValueError("gemm_hnorm expects bf16 operands and norm weight")
    if a.dim() != 2 or w.dim() != 2 or a.shape[1] != w.shape[1] or a.stride(1) != 1 or w.stride(1) != 1:
        raise ValueError(f"gemm_hnorm shapes a{tuple(a.shape)} w{tuple(w.shape)}: need [M, K] x [N, K], K contiguous")
    if norm_weight.numel() != 128 or not norm_weight.is_contiguous() or norm_weight.device != a.device:
        raise ValueError("gemm_hnorm: norm_weight must be a contiguous bf16 [128] device tensor")
    M, K = a.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if tuple(out.shape) != (M, N) or out.stride(1) != 1:
        raise ValueError(f"gemm_hnorm out {tuple(out.shape)} != ({M}, {N})")
    rc = lib.cp25_gemm_hnorm(_ptr(a), a.stride(0), _ptr(w), w.stride(0), _ptr(out), out.stride(0), M, N, K,
                             _ptr(norm_weight), float(eps), float(out_scale), _stream(a.device))
    if rc == -95:
        return None
    _check("cp25_gemm_hnorm", rc)
    return out


def gemm_qkv(a: torch.Tensor, w: torch.Tensor, k_norm_weight: torch.Tensor, *, k_col0: int, k_cols: int, B: int,
             cos: Optional[torch.Tensor] = None, sin: Optional[torch.Tensor] = None, eps: float = 1e-6,
             out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """The fused q|k|v projection out[M, N] = bf16(a w^T) with the k columns [k_col0, k_col0 + k_cols) normalised per
    128-column head (k_norm_weight, eps) and rotated by the RoPE of token row // B (cos / sin [M / B, 64] fp32 or None)
    in the epilogue (cp25_gemm_qkv): bit-identical to gemm_epi + head_rmsnorm_rope on those columns. None when the
    kernel is not built for the shape (K / 64 odd): the caller runs the two ops."""
    lib = load_library()
    if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or k_norm_weight.dtype != torch.bfloat16:
        raise ValueError("gemm_qkv expects bf16 operands and norm weight")
    if a.dim() != 2 or w.dim() != 2 or a.shape[1] != w.shape[1] or a.stride(1) != 1 or w.stride(1) != 1:
        raise ValueError(f"gemm_qkv shapes a{tuple(a.shape)} w{tuple(w.shape)}: need [M, K] x [N, K], K contiguous")
    if k_norm_weight.numel() != 128 or not k_norm_weight.is_contiguous() or k_norm_weight.device != a.device:
        raise ValueError("gemm_qkv: k_norm_weight must be a contiguous bf16 [128] device tensor")
    M, K = a.shape
    N = w.shape[0]
    if (cos is None) != (sin is None):
        raise ValueError("gemm_qkv: cos and sin go together")
    if cos is not None:
        for t in (cos, sin):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.dim() != 2 or t.shape[1] != 64 or \
                    t.shape[0] * B < M or t.device != a.device:
                raise ValueError(f"gemm_qkv: cos/sin must be contiguous float32 [>= {M // B}, 64] device tables")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if tuple(out.shape) != (M, N) or out.stride(1) != 1:
        raise ValueError(f"gemm_qkv out {tuple(out.shape)} != ({M}, {N})")
    rc = lib.cp25_gemm_qkv(_ptr(a), a.stride(0), _ptr(w), w.stride(0), _ptr(out), out.stride(0), M, N, K, int(k_col0),
                           int(k_cols), _ptr(k_norm_weight), _ptr(cos), _ptr(sin), int(B), float(eps),
                           _stream(a.device))
    if rc == -95:
        return None
    _check("cp25_gemm_qkv", rc)
    return out


def gemm_res(a: torch.Tensor, w: torch.Tensor, x: torch.Tensor, x_st: int, x_sb: int, gate: torch.Tensor, *, B: int,
             tok0: int, hw: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[M, N] = bf16(x + bf16(gate * bf16(a[M, K] w[N, K]^T))) (cp25_gemm_res): the block's gated residual fused into
    the projection. Row r of out / a is token r // B, batch entry r % B; x is read as x[tok * x_st + b * x_sb + col]
    (x_sb = 0 broadcasts one row), gate is a bf16 [B', T, N] view (strides (sb, st, 1)) read at the row's frame
    (tok0 + tok) // hw."""
    lib = load_library()
    if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or gate.dtype != torch.bfloat16:
        raise ValueError("gemm_res expects bf16 operands")
    if a.dim() != 2 or w.dim() != 2 or a.shape[1] != w.shape[1] or a.stride(1) != 1 or w.stride(1) != 1:
        raise ValueError(f"gemm_res shapes a{tuple(a.shape)} w{tuple(w.shape)}: need [M, K] x [N, K], K contiguous")
    M, K = a.shape
    N = w.shape[0]
    if gate.dim() != 3 or gate.shape[-1] != N or gate.stride(2) != 1 or gate.shape[0] < B:
        raise ValueError(f"gemm_res gate {tuple(gate.shape)}: need a [B, T, {N}] view with a unit inner stride")
    n_tok = M // B
    _check_frames(gate, n_tok=n_tok, B=B, tok0=tok0, hw=hw)
    if M % B or x.stride(-1) != 1 or \
            (n_tok - 1) * x_st + (B - 1) * x_sb + N > x.untyped_storage().nbytes() // 2 - x.storage_offset():
        raise ValueError("gemm_res: x does not cover the rows")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if tuple(out.shape) != (M, N) or out.stride(1) != 1:
        raise ValueError(f"gemm_res out {tuple(out.shape)} != ({M}, {N})")
    rc = lib.cp25_gemm_res(_ptr(a), a.stride(0), _ptr(w), w.stride(0), _ptr(out), out.stride(0), M, N, K, _ptr(x), x_st,
                           x_sb, _ptr(gate), gate.stride(0), gate.stride(1), B, tok0, hw, _stream(a.device))
    _check("cp25_gemm_res", rc)
    return out


def gemm_fp8_supported(N: int, K: int) -> bool:
    """Shapes cp25_gemm_fp8 is built for (N multiple of 256, K of 256); the fp8 option raises ValueError for others."""
    return N % 256 == 0 and K % 256 == 0


def gemm_fp8(q: torch.Tensor, s: torch.Tensor, w8: torch.Tensor, ws: torch.Tensor, *, res=None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 (q[M, K] w8[N, K]^T) * s[m] * ws[n] on the hand-written fp8 GEMM (cp25_gemm_fp8: torch._scaled_mm's
    row / column-scaled definition). q, w8 float8_e4m3fn (K contiguous), s [M, 1] / ws [1, N] (or [N]) fp32.
    res = (x, x_st, x_sb, gate, B, tok0, hw): the gated-residual epilogue of gemm_res (cp25_gemm_fp8_res)."""
    lib = load_library()
    if q.dtype != torch.float8_e4m3fn or w8.dtype != torch.float8_e4m3fn:
        raise ValueError("gemm_fp8 expects float8_e4m3fn operands")
    if q.dim() != 2 or w8.dim() != 2 or q.shape[1] != w8.shape[1] or q.stride(1) != 1 or w8.stride(1) != 1:
        raise ValueError(f"gemm_fp8 shapes q{tuple(q.shape)} w{tuple(w8.shape)}")
    M, K = q.shape
    Nn = w8.shape[0]
    if s.dtype != torch.float32 or ws.dtype != torch.float32 or s.numel() != M or ws.numel() != Nn or \
            not s.is_contiguous() or not ws.is_contiguous():
        raise ValueError("gemm_fp8 scales: contiguous fp32 [M] rows and [N] columns")
    if out is None:
        out = torch.empty((M, Nn), dtype=torch.bfloat16, device=q.device)
    if tuple(out.shape) != (M, Nn) or out.stride(1) != 1 or out.dtype != torch.bfloat16:
        raise ValueError(f"gemm_fp8 out {tuple(out.shape)} != ({M}, {Nn})")
    if res is None:
        rc = lib.cp25_gemm_fp8(_ptr(q), q.stride(0), _ptr(s), _ptr(w8), w8.stride(0), _ptr(ws), _ptr(out), out.stride(0),
                               M, Nn, K, _stream(q.device))
        _check("cp25_gemm_fp8", rc)
        return out
    x, x_st, x_sb, gate, B, tok0, hw = res
    if x.dtype != torch.bfloat16 or gate.dtype != torch.bfloat16 or gate.dim() != 3 or gate.stride(2) != 1:
        raise ValueError("gemm_fp8 res: bf16 x and a [B, T, N] bf16 gate view")
    _check_frames(gate, n_tok=M // B, B=B, tok0=tok0, hw=hw)
    rc = lib.cp25_gemm_fp8_res(_ptr(q), q.stride(0), _ptr(s), _ptr(w8), w8.stride(0), _ptr(ws), _ptr(out),
                               out.stride(0), M, Nn, K, _ptr(x), x_st, x_sb, _ptr(gate), gate.stride(0), gate.stride(1),
                               B, tok0, hw, _stream(q.device))
    _check("cp25_gemm_fp8_res", rc)
    return out


def quant_fp8_rows(x: torch.Tensor, gelu: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-scaled fp8 (float8_e4m3fn) operand of x [M, K] bf16: returns (q [M, K], scale [M, 1] fp32) with
    x ~= q * scale (of GELU(x) when gelu=True). cp25_quant_fp8_rows / cp25_gelu_quant_fp8."""
    lib = load_library()
    if x.dim() != 2 or not x.is_contiguous() or x.dtype != torch.bfloat16:
        raise ValueError("quant_fp8_rows expects a contiguous 2-D bf16 tensor")
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.empty((x.shape[0], 1), dtype=torch.float32, device=x.device)
    fn = lib.cp25_gelu_quant_fp8 if gelu else lib.cp25_quant_fp8_rows
    _check("cp25_gelu_quant_fp8" if gelu else "cp25_quant_fp8_rows",
           fn(_ptr(x), _ptr(q), _ptr(s), x.shape[0], x.shape[1], _stream(x.device)))
    return q, s


def patchify(xs: torch.Tensor, gt: Optional[torch.Tensor], frame_mask: torch.Tensor,
             pad_mask: Optional[torch.Tensor], *, tok0: int, hw: int, ld: int = 72) -> torch.Tensor:
    """x_embedder input rows [n_tok, 72] bf16 (cp25_patchify). ld = 128: the rows live in a zero-padded
    [n_tok, 128] buffer (cp25_patchify_ld) and the returned [n_tok, 72] view has row stride 128, the own GEMM's
    K = 128 operand (DiT.embed_patches)."""
    lib = load_library()
    n_tok = xs.shape[0]
    _check_mask(frame_mask, n_tok=n_tok, tok0=tok0, hw=hw)
    out = torch.empty((n_tok, ld), dtype=torch.bfloat16, device=xs.device)
    if ld == 72:
        rc = lib.cp25_patchify(_ptr(xs), _ptr(gt), _ptr(frame_mask), _ptr(pad_mask), _ptr(out), n_tok, tok0, hw,
                               _stream(xs.device))
    else:
        rc = lib.cp25_patchify_ld(_ptr(xs), _ptr(gt), _ptr(frame_mask), _ptr(pad_mask), _ptr(out), int(ld), n_tok,
                                  tok0, hw, _stream(xs.device))
    _check("cp25_patchify", rc)
    return out[:, :72]


def cfg_velocity(net: torch.Tensor, noise: Optional[torch.Tensor], gt: Optional[torch.Tensor],
                 frame_mask: Optional[torch.Tensor], guidance: float, cfg_mode: int, *, tok0: int,
                 hw: int) -> torch.Tensor:
    lib = load_library()
    n_tok, B, _ = net.shape
    if frame_mask is not None:
        _check_mask(frame_mask, n_tok=n_tok, tok0=tok0, hw=hw)
    out = torch.empty((n_tok, 64), dtype=torch.float32, device=net.device)
    rc = lib.cp25_cfg_velocity(_ptr(net), B, _ptr(noise), _ptr(gt), _ptr(frame_mask), float(guidance), int(cfg_mode),
                               _ptr(out), n_tok, tok0, hw, _stream(net.device))
    _check("cp25_cfg_velocity", rc)
    return out


def unipc_step(x: torch.Tensor, v: torch.Tensor, m0: torch.Tensor, m1: torch.Tensor, last: torch.Tensor,
               params: UniPCParams) -> None:
    lib = load_library()
    for t in (x, v, m0, m1, last):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != x.numel():
            raise ValueError("unipc_step expects contiguous fp32 tensors of equal size")
    rc = lib.cp25_unipc_step(_ptr(x), _ptr(v), _ptr(m0), _ptr(m1), _ptr(last), x.numel(), ctypes.byref(params),
                             _stream(x.device))
    _check("cp25_unipc_step", rc)


# ----------------------------------------------------------------------------- VAE
def conv3d(frames, weight: torch.Tensor, bias: Optional[torch.Tensor], out: torch.Tensor, *, Hin: int, Win: int,
           Cin: int, Cout: int, Tout: int, KT: int, KH: int, KW: int, stride_t: int = 1, stride_hw: int = 1,
           pad: tuple = (0, 0, 0, 0), upsample: bool = False, out_split: int = 0,
           residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Implicit-GEMM causal conv (see include/cp25.h). frames: list of channels-last frame tensors
    (or None for a zero frame); weight [Cout, KT, KH, KW, Cin] bf16; pad = (top, left, bottom, right)."""
    lib = load_library()
    ptrs = (ctypes.c_void_p * len(frames))(*[(_ptr(f) if f is not None else None) for f in frames])
    dev = out.device
    rc = lib.cp25_conv3d(ptrs, len(frames), _ptr(weight), _ptr(bias), _ptr(residual), _ptr(out), Hin, Win, Cin, Cout,
                         Tout, KT, KH, KW, stride_t, stride_hw, pad[0], pad[1], pad[2], pad[3], int(upsample),
                         out_split, _stream(dev))
    _check("cp25_conv3d", rc)
    return out


def conv3d_select(mode: int) -> int:
    """cp25_conv3d_select: 0 = the halo kernel for 3x3 stride-1 convs (default), 1 = the per-tap kernel everywhere
    (A/B and tests). Returns the previous mode."""
    rc = load_library().cp25_conv3d_select(int(mode))
    _check("cp25_conv3d_select", min(rc, 0))
    return rc


def rms_norm_silu(x: torch.Tensor, gamma: torch.Tensor, silu: bool = True, out: Optional[torch.Tensor] = None):
    lib = load_library()
    C = x.shape[-1]
    if out is None:
        out = torch.empty_like(x)
    if not x.is_contiguous():
        raise ValueError("rms_norm_silu expects a contiguous channels-last tensor")
    rc = lib.cp25_rms_norm_silu(_ptr(x), _ptr(gamma), _ptr(out), x.numel() // C, C, int(silu), _stream(x.device))
    _check("cp25_rms_norm_silu", rc)
    return out


def vae_attn(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: Optional[torch.Tensor] = None,
             scale: Optional[float] = None) -> torch.Tensor:
    """Single-head attention per frame for the VAE AttentionBlock (cp25_vae_attn): q [T, Lq, 384], k / v
    [T, Lk, 384] bf16 views with unit inner stride (e.g. column slices of the to_qkv output) -> out [T, Lq, 384]."""
    lib = load_library()
    for n, t in (("q", q), ("k", k), ("v", v)):
        if t.dtype != torch.bfloat16 or t.dim() != 3 or t.stride(2) != 1 or t.device != q.device:
            raise ValueError(f"vae_attn: {n} must be a [T, L, D] bf16 view with unit inner stride")
    T, Lq, D = q.shape
    if k.shape[0] != T or v.shape[0] != T or k.shape[2] != D or v.shape[2] != D or v.shape[1] != k.shape[1]:
        raise ValueError("vae_attn: q / k / v shapes disagree")
    if out is None:
        out = torch.empty((T, Lq, D), dtype=torch.bfloat16, device=q.device)
    if out.shape != q.shape or out.dtype != torch.bfloat16 or out.stride(2) != 1:
        raise ValueError("vae_attn: out must be a [T, Lq, D] bf16 tensor with unit inner stride")
    sc = D ** -0.5 if scale is None else float(scale)
    nbytes = lib.cp25_vae_attn_workspace_bytes(T, Lq, k.shape[1], D)
    ws = torch.empty((max(nbytes, 0) + 3) // 4, dtype=torch.float32, device=q.device) if nbytes > 0 else None
    rc = lib.cp25_vae_attn(_ptr(q), q.stride(1), q.stride(0), _ptr(k), k.stride(1), k.stride(0), _ptr(v), v.stride(1),
                           v.stride(0), _ptr(out), out.stride(1), out.stride(0), T, Lq, k.shape[1], D, sc, _ptr(ws),
                           max(nbytes, 0), _stream(q.device))
    _check("cp25_vae_attn", rc)
    return out


def softmax_rows(s: torch.Tensor, scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 softmax(s * scale) over the last dim of a 2-D fp32 score matrix (cp25_softmax_rows)."""
    lib = load_library()
    if s.dtype != torch.float32 or s.dim() != 2 or s.stride(1) != 1:
        raise ValueError("softmax_rows expects a row-major 2-D fp32 tensor")
    rows, cols = s.shape
    if out is None:
        out = torch.empty((rows, cols), dtype=torch.bfloat16, device=s.device)
    if out.shape != s.shape or out.dtype != torch.bfloat16 or out.stride(1) != 1:
        raise ValueError("softmax_rows: out must be a row-major bf16 tensor of the same shape")
    rc = lib.cp25_softmax_rows(_ptr(s), rows, cols, s.stride(0), float(scale), _ptr(out), out.stride(0),
                               _stream(s.device))
    _check("cp25_softmax_rows", rc)
    return out
