"""CPU: the autoregressive sliding window (Video2WorldInference.generate_autoregressive_from_batch) is
byte-identical to the oracle restatement of video2world.py:582-810, with a stand-in denoiser in place of
generate_vid2world (the window is host logic: chunk slicing, padding, uint8 re-quantisation, seeds)."""
import pytest
import torch

import __graft_entry__  # noqa: F401  (sets sys.path)
from cosmos_predict2.pipeline import Video2WorldInference
from oracle.ar_window import autoregressive, chunk_plan

H, W = 8, 12


def stand_in(chunk_u8: torch.Tensor, num_cond: int, seed: int) -> torch.Tensor:
    """Deterministic 'model': fp32 video in (-1.3, 1.3) (exercises the clamp and the truncation), a
    function of every input byte, the conditioning count and the seed."""
    g = torch.Generator().manual_seed(1000 * seed + num_cond)
    x = chunk_u8.float() / 127.5 - 1.0
    mix = x.flip(2).roll(1, dims=3) * 0.7 + 0.6 * torch.sin(x * 3.0 + seed)
    return (mix + 0.05 * torch.randn(x.shape, generator=g)).float()


class _Rec:
    """Records every call so the conditioning inputs can be compared too."""

    def __init__(self):
        self.calls = []

    def __call__(self, chunk, num_cond, seed):
        self.calls.append((chunk.clone(), num_cond, seed))
        return stand_in(chunk, num_cond, seed)


def _pipe(model_frames: int, rec: _Rec):
    p = object.__new__(Video2WorldInference)

    class _Tok:
        @staticmethod
        def get_pixel_num_frames(t):
            return 1 + 4 * (t - 1)

    class _Cfg:
        state_t = 1 + (model_frames - 1) // 4
        resolution = "480"

    class _Model:
        tokenizer = _Tok()
        config = _Cfg()

    p.model = _Model()
    p.generate_vid2world = lambda prompt, inp, guidance, frames, ncond, res, seed, neg, steps: rec(inp, ncond, seed)
    return p


@pytest.mark.parametrize("n_out,chunk,overlap", [(29, 13, 1), (29, 13, 5), (40, 13, 5), (13, 13, 1), (9, 13, 1),
                                                 (57, 21, 5)])
def test_ar_window_byte_identical(n_out, chunk, overlap):
    model_frames = 13 if chunk <= 13 else 21
    g = torch.Generator().manual_seed(7)
    vid = torch.randint(0, 256, (1, 3, 1, H, W), generator=g, dtype=torch.uint8)  # image input: frame 0
    rec_p, rec_o = _Rec(), _Rec()
    got = _pipe(model_frames, rec_p).generate_autoregressive_from_batch(
        "p", vid, num_output_frames=n_out, chunk_size=chunk, chunk_overlap=overlap, num_latent_conditional_frames=1,
        resolution=f"{H},{W}", seed=3)
    ref = autoregressive(rec_o, vid, n_out, chunk, overlap, model_frames, 1, 3)
    assert len(rec_p.calls) == len(rec_o.calls) == len(chunk_plan(n_out, chunk, overlap))
    for (a, ca, sa), (b, cb, sb) in zip(rec_p.calls, rec_o.calls):
        assert a.dtype == torch.uint8 and torch.equal(a, b) and ca == cb and sa == sb
    assert got.dtype == ref.dtype and torch.equal(got, ref)
    assert got.shape[2] == n_out


def test_chunk_plan_ragged_last_chunk():
    # 40 frames, chunk 13, overlap 5: starts 0, 8, 16, 24, 32 -> the last chunk is [32, 40), 8 frames
    assert chunk_plan(40, 13, 5) == [(0, 13), (8, 21), (16, 29), (24, 37), (32, 40)]
    assert chunk_plan(13, 13, 1) == [(0, 13)]


def test_requantisation_truncates():
    # video2world.py:798 truncates; rounding would give 128 for v = 0.0039 (0.50196 * 255 = 127.998)
    v = torch.tensor([0.0039, -1.5, 1.5, 0.999], dtype=torch.float32)
    q = ((v / 2.0 + 0.5).clamp(0.0, 1.0) * 255.0).to(torch.uint8)
    assert q.tolist() == [127, 0, 255, 254]
