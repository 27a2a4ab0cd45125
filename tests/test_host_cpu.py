"""CPU: C-ABI exports, host-side math and layouts of the product (no kernel launches)."""
import ctypes
import dataclasses
import re

import numpy as np
import pytest
import torch

import __graft_entry__  # noqa: F401  (sets sys.path)
from cosmos_predict2 import _native
from cosmos_predict2.dit import init_state_dict, rope_freqs, state_dict_shapes
from cosmos_predict2.model import from_patch_layout, to_patch_layout
from cosmos_predict2.net_config import DIT_2B, DIT_14B, tiny_dit
from cosmos_predict2.scheduler import FlowUniPCMultistepScheduler
from cosmos_predict2.vae import vae_state_dict_shapes
from oracle import dit as odit
from oracle.unipc import UniPC, _coeffs


def test_library_exports_every_header_symbol():
    hdr = open(__graft_entry__.ROOT + "/include/cp25.h").read()
    # every function declaration at column 0, whatever its return type (int, int64_t, size_t, const char*)
    declared = sorted(set(re.findall(r"^(?:const\s+)?[A-Za-z_]\w*\s*\**\s*(cp25_\w+)\(", hdr, re.M)))
    assert len(declared) >= 48 and "cp25_gemm_epi_t" in declared and "cp25_gemm_f32_workspace_floats" in declared and "cp25_attn_kernel" in declared
    lib = _native.load_library()
    for name in declared:
        assert hasattr(lib, name), name
        assert name in _native.SIGNATURES, f"{name} has no ctypes signature"
    assert ctypes.sizeof(_native.UniPCParams) == 15 * 4


def test_host_rejects_cpu_tensors():
    with pytest.raises(RuntimeError):
        _native.attn_fwd(torch.zeros(1, 4, 1, 128, dtype=torch.bfloat16), torch.zeros(1, 4, 1, 128, dtype=torch.bfloat16),
                         torch.zeros(1, 4, 1, 128, dtype=torch.bfloat16))


@pytest.mark.parametrize("karras,n", [(True, 35), (False, 35), (True, 2), (False, 7)])
def test_scheduler_host_coefficients_match_oracle(karras, n):
    """The fused kernel's scalar coefficients equal the oracle's (reference op order, fp32) bit-exactly."""
    s = FlowUniPCMultistepScheduler(shift=1)
    s.set_timesteps(n, shift=5.0, use_kerras_sigma=karras)
    o = UniPC(n, shift=5.0, use_karras=karras)
    assert torch.equal(s.timesteps, o.timesteps) and torch.equal(s.sigmas, o.sigmas)
    s._step_index = 0
    for k in range(len(s.timesteps)):
        s._step_index = k
        s._have_last = k > 0
        s.lower_order_nums = min(k, 2)
        s.this_order = min(2, len(s.timesteps) - (k - 1), k) if k > 0 else None
        P, order = s._params()
        c = _coeffs(o.sigmas, k + 1, k, [k - 1], order)
        assert P.p_a == (c["sigma_t"] / c["sigma_s0"]).item()
        assert P.p_b == (c["alpha_t"] * c["h_phi_1"]).item()
        assert P.p_c == (c["alpha_t"] * c["B_h"]).item()
        if order == 2:
            assert P.p_inv_rk == (torch.tensor(1.0) / c["rks"][0]).item()


def test_patch_layout_roundtrip():
    x = torch.randn(16, 3, 8, 12)
    p = to_patch_layout(x)
    assert p.shape == (3 * 4 * 6, 64)
    # token (t, h2, w2), feature (p1*2 + p2)*16 + c
    assert p[1 * 24 + 2 * 6 + 3, (1 * 2 + 0) * 16 + 5] == x[5, 1, 2 * 2 + 1, 3 * 2 + 0]
    assert torch.equal(from_patch_layout(p, 3, 8, 12), x)


def test_dit_state_dict_layout_matches_reference():
    s = state_dict_shapes(DIT_2B)
    n = sum(np.prod(v[0]) for k, v in s.items() if not k.startswith("pos_embedder"))
    assert 2.0e9 < n < 2.1e9  # "~2.05 B params" 
    assert s["x_embedder.proj.1.weight"][0] == (2048, 72)
    assert s["crossattn_proj.0.weight"][0] == (1024, 100352)
    assert s["blocks.27.cross_attn.k_proj.weight"][0] == (2048, 1024)
    assert s["blocks.0.adaln_modulation_mlp.2.weight"][0] == (6144, 256)
    assert s["final_layer.linear.weight"][0] == (64, 2048)
    assert s["pos_embedder.dim_spatial_range"][0] == (21,) and s["pos_embedder.dim_temporal_range"][0] == (22,)
    s14 = state_dict_shapes(DIT_14B)
    assert sum(np.prod(v[0]) for v in s14.values()) > 1.3e10


def test_vae_state_dict_layout():
    s = vae_state_dict_shapes()
    n = sum(np.prod(v) for v in s.values())
    assert 1.2e8 < n < 1.3e8  # Wan2.1 VAE ~127 M
    assert s["decoder.upsamples.3.time_conv.weight"] == (768, 384, 3, 1, 1)
    assert s["encoder.downsamples.5.time_conv.weight"] == (192, 192, 3, 1, 1)
    assert s["decoder.head.2.weight"] == (3, 96, 3, 3, 3)


def test_rope_freqs_match_oracle():
    cfg = tiny_dit()
    sd = init_state_dict(cfg, seed=0)
    a = rope_freqs(cfg, 3, 4, 5, sd, "cpu")
    b = odit.rope_freqs(dataclasses.asdict(cfg), 3, 4, 5)
    assert torch.equal(a, b)


def test_inference_arguments_api():
    from cosmos_predict2.config import InferenceArguments, SetupArguments

    a = InferenceArguments(name="s", prompt="p", inference_type="text2world")
    assert a.num_steps == 35 and a.guidance == 7 and a.seed == 0 and a.num_input_frames == 0
    with pytest.raises(Exception):
        InferenceArguments(name="s", prompt="p", inference_type="image2world")  # input_path required
    s = SetupArguments(output_dir="/tmp/x")
    assert s.model == "2B/post-trained" and s.context_parallel_size >= 1


_LIBRARY_MATH = {"linear", "_scaled_mm", "matmul", "mm", "bmm", "addmm", "baddbmm", "einsum", "conv1d", "conv2d",
                 "conv3d", "scaled_dot_product_attention"}


def test_package_has_no_library_math():
    """No sampler or setup path falls back to a library GEMM / conv / attention: the package source
    calls none of torch / F's matrix ops, and has no tensor `@` outside action_conditioned.py's numpy 3 x 3 rotation
    math (host-side action preprocessing, reference data prep)."""
    import ast
    import os

    pkg = os.path.dirname(_native.__file__)
    found = []
    for fn in sorted(os.listdir(pkg)):
        if not fn.endswith(".py"):
            continue
        tree = ast.parse(open(os.path.join(pkg, fn)).read())
        for node in ast.walk(tree):
            if (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr in _LIBRARY_MATH
                    and isinstance(node.func.value, ast.Name) and node.func.value.id in ("F", "torch", "nn")):
                found.append(f"{fn}:{node.lineno} {node.func.value.id}.{node.func.attr}")
            if isinstance(node, ast.BinOp) and isinstance(node.op, ast.MatMult) and fn != "action_conditioned.py":
                found.append(f"{fn}:{node.lineno} @")
    assert not found, found


def test_unsupported_gemm_shape_raises():
    """A projection weight the own GEMM is not built for raises ValueError (no library fallback)."""
    from cosmos_predict2.dit import _require_gemm

    _require_gemm(torch.empty(512, 384))
    for shape in ((500, 384), (512, 100)):
        with pytest.raises(ValueError):
            _require_gemm(torch.empty(*shape))


def _desc(dtype, shape, strides=None, data=0x100000):
    """A cp25_tensor with a fake (never dereferenced) device address: the checks below fail before any GPU work."""
    d = _native.CP25Tensor()
    d.data, d.dtype, d.ndim = data, dtype, len(shape)
    if strides is None:
        strides, acc = [], 1
        for n in reversed(shape):
            strides.insert(0, acc)
            acc *= n
    for i, (n, st) in enumerate(zip(shape, strides)):
        d.shape[i], d.strides[i] = n, st
    return d


def test_descriptor_abi_rejects_bad_dtypes_and_strides():
    """the descriptor entry points return CP25_ERR_DTYPE (-95) for a wrong dtype
    and CP25_ERR_INVAL (-22) for a shape / stride / pointer mismatch on the host, before anything touches a GPU (this
    machine has none, so reaching a launch would fail differently)."""
    lib = _native.load_library()
    bf, f32 = _native.DT_BF16, _native.DT_F32
    r = ctypes.byref
    # attention: q fp32 where bf16 is required
    q, k, v, o = (_desc(bf, (1, 300, 2, 128)) for _ in range(4))
    assert lib.cp25_attn_fwd_t(r(_desc(f32, (1, 300, 2, 128))), r(k), r(v), r(o), 0.1, None, 0, None) == -95
    assert lib.cp25_attn_fwd_t(r(q), r(k), r(_desc(_native.DT_F8E4M3, (1, 300, 2, 128))), r(o), 0.1, None, 0, None) == -95
    assert lib.cp25_attn_fwd_t(r(q), r(k), r(v), r(_desc(bf, (1, 300, 2, 128), (76800, 256, 128, 2))), 0.1, None, 0,
                               None) == -22  # head dim not contiguous
    assert lib.cp25_attn_fwd_t(r(q), r(_desc(bf, (1, 299, 2, 128))), r(v), r(o), 0.1, None, 0, None) == -22  # k vs v
    assert lib.cp25_attn_fwd_t(r(_desc(bf, (1, 300, 2, 64))), r(_desc(bf, (1, 300, 2, 64))), r(_desc(bf, (1, 300, 2, 64))),
                               r(_desc(bf, (1, 300, 2, 64))), 0.1, None, 0, None) == -95  # head dim 64
    assert lib.cp25_attn_fwd_t(None, r(k), r(v), r(o), 0.1, None, 0, None) == -22
    # GEMM
    a, w, c = _desc(bf, (512, 256)), _desc(bf, (256, 256)), _desc(bf, (512, 256))
    assert lib.cp25_gemm_epi_t(r(_desc(f32, (512, 256))), r(w), r(c), 0, None) == -95
    assert lib.cp25_gemm_epi_t(r(a), r(w), r(_desc(f32, (512, 256))), 0, None) == -95
    assert lib.cp25_gemm_epi_t(r(a), r(_desc(bf, (256, 128))), r(c), 0, None) == -22  # K mismatch
    assert lib.cp25_gemm_epi_t(r(a), r(w), r(_desc(bf, (512, 256), (1, 512))), 0, None) == -22  # column-major c
    assert lib.cp25_gemm_epi_t(r(a), r(w), r(c), 2, None) == -22  # the residual epilogue needs its operands
    assert lib.cp25_gemm_epi_t(r(_desc(bf, (512, 256), data=0)), r(w), r(c), 0, None) == -22  # null pointer
    # conv
    x, wt, b, out = _desc(bf, (4, 8, 8, 16)), _desc(bf, (32, 3, 3, 3, 16)), _desc(bf, (32,)), _desc(bf, (4, 8, 8, 32))
    assert lib.cp25_conv3d_t(r(_desc(f32, (4, 8, 8, 16))), 2, r(wt), r(b), r(out), 1, 1, 1, 1, 1, 1, None) == -95
    assert lib.cp25_conv3d_t(r(x), 2, r(wt), r(_desc(f32, (32,))), r(out), 1, 1, 1, 1, 1, 1, None) == -95
    assert lib.cp25_conv3d_t(r(x), 2, r(wt), r(b), r(_desc(bf, (4, 8, 8, 31))), 1, 1, 1, 1, 1, 1, None) == -22
    assert lib.cp25_conv3d_t(r(x), 0, r(wt), r(b), r(out), 1, 1, 1, 1, 1, 1, None) == -22  # too few frames for KT = 3
    assert lib.cp25_conv3d_t(r(x), 2, r(wt), r(b), r(_desc(bf, (4, 7, 8, 32))), 1, 1, 1, 1, 1, 1, None) == -22  # Ho


def test_tensor_desc_of_a_torch_tensor():
    t = torch.zeros(3, 5, 7, dtype=torch.bfloat16)[:, 1:4]
    with pytest.raises(RuntimeError):  # host tensors are refused like every other binding
        _native.tensor_desc(t)
    assert ctypes.sizeof(_native.CP25Tensor) == 8 + 4 + 4 + 6 * 8 * 2
