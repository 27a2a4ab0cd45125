"""Host side of the action-conditioned chunk loop: the conditioning video of a chunk equals the reference's
construction (cosmos_predict2/action_conditioned.py:326-331: to_tensor -> zero frames -> * 255 -> uint8), restated
here in fp32 torch, on every uint8 value and on a random frame."""
import numpy as np
import torch

import __graft_entry__  # noqa: F401  (import paths)
from cosmos_predict2.action_conditioned import conditioning_video


def _reference_form(img: np.ndarray, n_frames: int) -> torch.Tensor:
    x = torch.from_numpy(np.ascontiguousarray(img.transpose(2, 0, 1))).float().div(255)[None]  # to_tensor
    vid = torch.cat([x, torch.zeros_like(x).repeat(n_frames - 1, 1, 1, 1)], 0)
    return (vid * 255.0).to(torch.uint8).unsqueeze(0).permute(0, 2, 1, 3, 4)


def test_conditioning_video_matches_reference_round_trip():
    every = np.arange(256, dtype=np.uint8).reshape(16, 16, 1).repeat(3, 2)
    assert torch.equal(conditioning_video(every, 13), _reference_form(every, 13))
    img = np.random.RandomState(0).randint(0, 256, size=(48, 64, 3), dtype=np.uint8)
    v = conditioning_video(img, 13)
    assert v.dtype == torch.uint8 and v.shape == (1, 3, 13, 48, 64)
    assert torch.equal(v, _reference_form(img, 13))
