"""Action-conditioned autoregressive generation on the device (tiny ActionChunk net, real Wan VAE
layout with seeded weights): the chunk loop of the reference's action_conditioned.py:291-366."""
import numpy as np
import pytest
import torch

from cosmos_predict2.action_conditioned import ActionConditionedInference
from cosmos_predict2.net_config import tiny_dit
from cosmos_predict2.pipeline import Video2WorldInference

pytestmark = pytest.mark.gpu


def test_action_chunk_loop(device):
    cfg = tiny_dit(num_blocks=1, action_dim=7, action_per_latent_frame=4)
    pipe = Video2WorldInference("2B/robot/action-cond", device=device, net_cfg=cfg)
    ac = ActionConditionedInference(pipe)
    rng = np.random.RandomState(0)
    img = rng.randint(0, 256, size=(64, 80, 3), dtype=np.uint8)
    acts = rng.randn(30, 7).astype(np.float32)
    v = ac.generate(img, acts, chunk_size=12, num_steps=2, guidance=7)
    assert v.dtype == np.uint8 and v.shape == (13 + 12 + 12, 64, 80, 3)
    v2 = ac.generate(img, acts, chunk_size=12, num_steps=2, guidance=7, single_chunk=True)
    assert v2.shape == (13, 64, 80, 3)
    assert np.array_equal(v2, v[:13])  # deterministic (seeded noise per chunk)
    v3 = ac.generate(img, acts * 0 + 3.0, chunk_size=12, num_steps=2, guidance=7, single_chunk=True)
    assert not np.array_equal(v3, v2)  # the actions condition the output
