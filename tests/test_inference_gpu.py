"""The reference's user API end to end on the device (cosmos_predict2/inference.py:30-171):
Inference(SetupArguments).generate([InferenceArguments], output_dir) with the real 2B layout
(seeded random weights) at a tiny geometry, writing .mp4 like the reference, and Video2World taking
that .mp4 back as its input (video2world.py:150-233)."""
from pathlib import Path

import numpy as np
import pytest

from cosmos_predict2.config import InferenceArguments, SetupArguments
from cosmos_predict2.inference import Inference
from cosmos_predict2.video_io import read_mp4

pytestmark = pytest.mark.gpu


def test_inference_api_image_then_video2world(device, tmp_path):
    from PIL import Image

    img = np.random.RandomState(0).randint(0, 256, size=(96, 160, 3), dtype=np.uint8)
    Image.fromarray(img).save(tmp_path / "in.png")
    out = tmp_path / "out"
    inf = Inference(SetupArguments(output_dir=out, model="2B/post-trained", state_t=2, keep_going=False))
    common = dict(prompt="A robot arm stacks two cubes.", resolution="64,128", num_output_frames=5, num_steps=2,
                  guidance=3)
    paths = inf.generate([InferenceArguments(name="i2w", inference_type="image2world", input_path=tmp_path / "in.png",
                                             **common)], out)
    assert len(paths) == 1 and paths[0].endswith(".mp4")
    v = read_mp4(paths[0])
    assert v.shape == (5, 64, 128, 3) and v.dtype == np.uint8
    assert (out / "i2w.json").exists()
    paths2 = inf.generate([InferenceArguments(name="v2w", inference_type="video2world", input_path=Path(paths[0]),
                                              **common)], out)
    v2 = read_mp4(paths2[0])
    assert v2.shape == (5, 64, 128, 3)
    # deterministic: the same sample again gives the same file
    paths3 = inf.generate([InferenceArguments(name="i2w_again", inference_type="image2world",
                                              input_path=tmp_path / "in.png", **common)], out)
    assert np.array_equal(read_mp4(paths3[0]), v)
