"""The descriptor entry points (cp25_attn_fwd_t, cp25_gemm_epi_t, cp25_conv3d_t; SURVEY.md §8(b)5's cp25_tensor form)
against the pointer entry points they forward to: bit-identical outputs on the same inputs, and a wrong dtype or
stride raised as ValueError from the library's own check (tests/test_host_cpu.py checks the return codes without a
GPU). Reference ops: networks/attention.py:90-181, the block nn.Linear layers (minimal_v4_dit.py:227-254) and
CausalConv3d.forward (tokenizers/wan2pt1.py:44-62)."""
import pytest
import torch

from cosmos_predict2 import _native as N

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


@pytest.mark.parametrize("B,H,Lq,Lk", [(1, 2, 300, 700), (2, 3, 1000, 5000)])
def test_attn_fwd_t_matches_pointer_form(device, B, H, Lq, Lk):
    g = torch.Generator(device=device).manual_seed(Lq + Lk)
    q = torch.randn(B, Lq, H, 128, device=device, generator=g).to(BF16)
    kv = torch.randn(B, Lk, 2, H, 128, device=device, generator=g).to(BF16)
    k, v = kv[:, :, 0], kv[:, :, 1]  # strided views, unit head-dim stride
    ref = N.attn_fwd(q, k, v, softmax_scale=128 ** -0.5, n_split=1)
    o = torch.empty_like(q)
    N.attn_fwd_t(q, k, v, o, 128 ** -0.5)
    assert torch.equal(o, ref)
    n_split = N.attn_plan(B, H, Lq, Lk)
    ws = torch.empty(max(16, N.load_library().cp25_attn_workspace_bytes(B, H, Lq, n_split)), dtype=torch.uint8,
                     device=device)
    o2 = torch.empty_like(q)
    N.attn_fwd_t(q, k, v, o2, 128 ** -0.5, workspace=ws)
    assert torch.equal(o2, N.attn_fwd(q, k, v, softmax_scale=128 ** -0.5, n_split=n_split))
    with pytest.raises(ValueError):
        N.attn_fwd_t(q.float(), k, v, o, 128 ** -0.5)


def test_gemm_epi_t_matches_pointer_form(device):
    g = torch.Generator(device=device).manual_seed(3)
    a = torch.randn(1000, 2048, device=device, generator=g).to(BF16)
    w = (torch.randn(512, 2048, device=device, generator=g) * 2048 ** -0.5).to(BF16)
    c = torch.empty(1000, 768, device=device, dtype=BF16)[:, 128:640]  # a strided output view
    for epi in (N.EPI_NONE, N.EPI_GELU):
        N.gemm_epi_t(a, w, c, epi)
        assert torch.equal(c, N.gemm_epi(a, w, epilogue=epi))
    with pytest.raises(ValueError):
        N.gemm_epi_t(a, w.float(), c)
    with pytest.raises(ValueError):
        N.gemm_epi_t(a, w, torch.empty(768, 1000, device=device, dtype=BF16).t()[:, :512])  # column-major output


def test_conv3d_t_matches_pointer_form(device):
    g = torch.Generator(device=device).manual_seed(5)
    T, H, W, C, Co = 3, 10, 64, 96, 96
    x = torch.randn(T, H, W, C, device=device, generator=g).to(BF16)
    w = (torch.randn(Co, 3, 3, 3, C, device=device, generator=g) / (27 * C) ** 0.5).to(BF16)
    b = (0.1 * torch.randn(Co, device=device, generator=g)).to(BF16)
    ref = torch.empty(T, H, W, Co, device=device, dtype=BF16)
    N.conv3d([None, None, x[0], x[1], x[2]], w, b, ref, Hin=H, Win=W, Cin=C, Cout=Co, Tout=T, KT=3, KH=3, KW=3,
             pad=(1, 1, 1, 1))
    out = torch.empty_like(ref)
    N.conv3d_t(x, w, b, out, pad_front=2, pad=(1, 1, 1, 1))
    assert torch.equal(out, ref)
    with pytest.raises(ValueError):
        N.conv3d_t(x.float(), w, b, out, pad_front=2, pad=(1, 1, 1, 1))
    with pytest.raises(ValueError):
        N.conv3d_t(x, w, b, out[:, :-1], pad_front=2, pad=(1, 1, 1, 1))  # output height does not match the conv
