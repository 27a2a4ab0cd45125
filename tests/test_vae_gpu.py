"""Wan2.1 VAE parity: HIP implicit-GEMM conv path vs the CPU oracle (oracle/vae.py) on seeded weights.

Single convolution: the kernel accumulates in fp32 like cuDNN; tolerance rel-L2 <= 2e-3 (bf16 output
rounding + accumulation order). Full encode / decode stacks ~30 bf16 convolutions and norms; the
tolerance is rel-L2 <= 2e-2 (bf16 rounding flips compound through the stack), measured values are
printed and recorded in DESIGN.md.
"""
import pytest
import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N
from cosmos_predict2.vae import Wan2pt1VAEInterface, _Conv, init_vae_state_dict
from oracle import vae as ovae

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("cin,cout,k,stride,up", [(96, 96, 3, 1, False), (16, 384, 3, 1, False),
                                                  (192, 96, 3, 1, True), (96, 96, 3, 2, False),
                                                  (384, 1152, 1, 1, False), (96, 3, 3, 1, False)])
def test_conv2d_like(device, cin, cout, k, stride, up):
    g = torch.Generator().manual_seed(cin + cout)
    H, W = 12, 20
    x = torch.randn(1, cin, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(torch.bfloat16)
    b = (0.1 * torch.randn(cout, generator=g)).to(torch.bfloat16)
    xi = F.interpolate(x.float(), scale_factor=2.0, mode="nearest-exact") if up else x.float()
    if stride == 2:
        ref = F.conv2d(F.pad(xi, (0, 1, 0, 1)), w.float(), b.float(), stride=2)
    else:
        ref = F.conv2d(xi, w.float(), b.float(), padding=k // 2)
    ref = ref.to(torch.bfloat16)
    conv = _Conv(w, b, device)
    xl = x[0].permute(1, 2, 0).contiguous().to(device)  # [H, W, C]
    pad = (0, 0, 1, 1) if stride == 2 else (k // 2,) * 4
    out = conv([xl], 1, H, W, stride_hw=stride, pad=pad, upsample=up)
    err = rel_l2(out[0].permute(2, 0, 1).cpu(), ref[0])
    assert err <= 2e-3, err


def test_causal_conv3d_with_cache(device):
    """3x3x3 causal conv over [cache(2 frames) | x(3 frames)] vs F.conv3d on the concatenated clip."""
    g = torch.Generator().manual_seed(5)
    C, H, W = 96, 10, 14
    cache = torch.randn(1, C, 2, H, W, generator=g).to(torch.bfloat16)
    x = torch.randn(1, C, 3, H, W, generator=g).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, 3, generator=g) / (27 * C) ** 0.5).to(torch.bfloat16)
    b = (0.1 * torch.randn(C, generator=g)).to(torch.bfloat16)
    ref = F.conv3d(F.pad(torch.cat([cache, x], 2).float(), (1, 1, 1, 1, 0, 0)), w.float(), b.float()).to(torch.bfloat16)
    conv = _Conv(w, b, device)
    cl = cache[0].permute(1, 2, 3, 0).contiguous().to(device)
    xl = x[0].permute(1, 2, 3, 0).contiguous().to(device)
    out = conv([cl[0], cl[1], xl[0], xl[1], xl[2]], 3, H, W, pad=(1, 1, 1, 1))
    assert rel_l2(out.permute(3, 0, 1, 2).cpu(), ref[0]) <= 2e-3


def test_rms_norm_silu(device):
    g = torch.Generator().manual_seed(6)
    x = torch.randn(1, 192, 3, 5, 7, generator=g).to(torch.bfloat16)
    gamma = (1 + 0.1 * torch.randn(192, 1, 1, 1, generator=g)).to(torch.bfloat16)
    ref = ovae.silu(ovae.rms_norm(x, gamma))
    out = N.rms_norm_silu(x[0].permute(1, 2, 3, 0).contiguous().to(device), gamma.reshape(-1).to(device))
    o = out.permute(3, 0, 1, 2).cpu()
    assert (o.float() - ref[0].float()).abs().max().item() <= 2 * 2 ** -7 * ref.float().abs().max().item()
    assert (o == ref[0]).float().mean().item() >= 0.99


@pytest.mark.parametrize("rows,cols", [(7, 5), (64, 1000), (3, 14080), (5, 4099)])
def test_softmax_rows(device, rows, cols):
    """AttentionBlock softmax (cp25_softmax_rows): fp32 scores -> bf16 P, within one bf16 rounding of
    torch.softmax in fp32; rows sum to 1 up to that rounding."""
    g = torch.Generator().manual_seed(rows + cols)
    s = (6 * torch.randn(rows, cols, generator=g)).to(device)
    scale = 384 ** -0.5
    p = N.softmax_rows(s, scale)
    ref = torch.softmax(s * scale, -1)
    assert p.dtype == torch.bfloat16
    assert ((p.float() - ref).abs() <= 2 ** -8 * ref + 1e-30).all()
    assert ((p.float().sum(-1) - 1).abs() <= 4e-3).all()
    with pytest.raises(ValueError):
        N.softmax_rows(s.to(torch.bfloat16), scale)


@pytest.fixture(scope="module")
def vae_pair():
    sd = init_vae_state_dict(seed=0)
    return sd


def _report(name, hip, ref, truth):
    d = dict(hip_truth=rel_l2(hip, truth), ref_truth=rel_l2(ref, truth), hip_ref=rel_l2(hip, ref))
    print(f"{name}: hip-vs-truth {d['hip_truth']:.3e}  bf16ref-vs-truth {d['ref_truth']:.3e}  "
          f"hip-vs-bf16ref {d['hip_ref']:.3e}")
    return d


def test_vae_encode_matches_oracle(device, vae_pair):
    """Encode (9 frames, 64 x 96) against the bf16 oracle and the fp32 truth (oracle.vae.fp32_truth: the same bf16
    weights, every activation fp32). The gate is the DiT's: the HIP path no further from the truth than the bf16
    reference restatement is (x 1.1); hip-vs-ref bounded by the measured value."""
    sd = vae_pair
    g = torch.Generator().manual_seed(7)
    video = (torch.rand(1, 3, 9, 64, 96, generator=g) * 2 - 1).to(torch.bfloat16)
    ref = ovae.encode(sd, video, temporal_window=4)
    with ovae.fp32_truth():
        truth = ovae.encode(sd, video, temporal_window=4)
    tok = Wan2pt1VAEInterface(sd, device=device, temporal_window=4)
    out = tok.encode(video.to(device))
    torch.cuda.synchronize()
    assert out.shape == ref.shape, (out.shape, ref.shape)
    d = _report("vae encode 9f 64x96", out.cpu(), ref, truth)
    # measured (MI355X, round 2): hip-vs-ref 7.6e-3
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 2e-2, d


def test_vae_decode_matches_oracle(device, vae_pair):
    """Decode of a 3 x 8 x 12 latent against the bf16 oracle and the fp32 truth (gate as for encode)."""
    sd = vae_pair
    g = torch.Generator().manual_seed(8)
    z = torch.randn(1, 16, 3, 8, 12, generator=g)
    ref = ovae.decode(sd, z)
    with ovae.fp32_truth():
        truth = ovae.decode(sd, z)
    tok = Wan2pt1VAEInterface(sd, device=device)
    out = tok.decode(z.to(device))
    torch.cuda.synchronize()
    assert out.shape == ref.shape, (out.shape, ref.shape)
    d = _report("vae decode 3x8x12", out.cpu(), ref, truth)
    # measured (MI355X, round 2): hip-vs-ref 1.3e-2
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 2e-2, d


def test_vae_decode_metric_geometry(device):
    """BASELINE config 2's decode geometry: 2 latent frames at 88 x 160 -> 5 frames at 704 x 1280
    (wan2pt1.py:551-570, WanVAE_.decode one latent frame at a time with the causal cache). The oracle at this size is
    ~4.5e13 FLOP (minutes on host cores), so the restatement runs on the GPU's own torch ops (fp32 MIOpen convs,
    fp32 matmuls), in bf16-reference mode and in fp32-truth mode; the HIP path (cp25_conv3d halo / per-tap convs,
    cp25_vae_attn, cp25_rms_norm_silu) must be as close to the truth as the bf16 reference is."""
    sd = init_vae_state_dict(seed=3)
    sdd = {k: v.to(device) for k, v in sd.items()}
    g = torch.Generator().manual_seed(12)
    z = torch.randn(1, 16, 2, 88, 160, generator=g).to(device)
    tok = Wan2pt1VAEInterface(sd, device=device)
    out = tok.decode(z)
    torch.cuda.synchronize()
    assert out.shape == (1, 3, 5, 704, 1280), out.shape
    def prog(i):
        torch.cuda.synchronize()
        print(f"  oracle decoded latent frame {i}", flush=True)

    # torch's own GPU convolutions without MIOpen (no per-shape kernel search / compile): im2col + fp32 GEMM
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False):
        ref = ovae.decode(sdd, z, progress=prog)
        with ovae.fp32_truth():
            truth = ovae.decode(sdd, z, progress=prog)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    d = _report("vae decode 2x88x160 -> 5f 704x1280", out.float(), ref.float(), truth.float())
    per_frame = [rel_l2(out[:, :, f].float(), ref[:, :, f].float()) for f in range(5)]
    print("  per output frame hip-vs-bf16ref: " + " ".join(f"{e:.2e}" for e in per_frame))
    assert d["hip_truth"] <= 1.1 * d["ref_truth"], d
    assert d["hip_ref"] <= 3e-2, d


def test_first_frame_encode_is_causal_prefix(device, vae_pair):
    """Latent frame 0 depends only on pixel frame 0: encoding the 1-frame prefix reproduces it
    bit-for-bit (this is what lets Image2World encode only the conditioning frame)."""
    sd = vae_pair
    g = torch.Generator().manual_seed(9)
    video = (torch.rand(1, 3, 9, 64, 96, generator=g) * 2 - 1).to(torch.bfloat16).to(device)
    tok = Wan2pt1VAEInterface(sd, device=device, temporal_window=4)
    full = tok.encode(video)
    first = tok.encode(video[:, :, :1])
    assert torch.equal(full[:, :, :1], first)


def _band_worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        vsd = init_vae_state_dict(seed=4)
        tok = Wan2pt1VAEInterface(vsd, device=dev)
        tok.set_context_parallel_group(dist.group.WORLD)
        z = torch.randn(1, 16, 3, 8, 12, generator=torch.Generator().manual_seed(8))
        q.put((rank, tok.decode(z.to(dev)).float().cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_decode_row_bands_match_full(device):
    """Context-parallel decode: two ranks (sharing cuda:0, gloo) each decode 4 of 8 latent rows with
    halo rows from the neighbour; the gathered video must equal the single-rank decode. Convs see
    identical inputs per output pixel (bit-exact); only the middle attention's fp32 GEMMs run at a
    different M, so the bound is rel-L2 <= 1e-3 (measured value printed)."""
    import socket

    import torch.multiprocessing as mp

    vsd = init_vae_state_dict(seed=4)
    tok = Wan2pt1VAEInterface(vsd, device=device)
    z = torch.randn(1, 16, 3, 8, 12, generator=torch.Generator().manual_seed(8))
    ref = tok.decode(z.to(device)).float().cpu()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_band_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: torch.from_numpy(a) for r, a in (q.get(timeout=100) for _ in ps)}
    for p in ps:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in ps)
    assert torch.equal(res[0], res[1])
    err = rel_l2(res[0], ref)
    print(f"banded decode (2 ranks) vs full decode rel-L2: {err:.3e}")
    assert err <= 1e-3, err
