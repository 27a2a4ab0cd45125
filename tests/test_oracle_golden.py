"""CPU: the oracle against the reference's recorded outputs and the committed golden vectors.

Pinning sources:
  * SURVEY.md F3 records what the reference's FlowUniPCMultistepScheduler.set_timesteps returned
    (fm_solvers_unipc.py:150-219): Karras 35 -> 36 int64 timesteps starting [995, 994, 993, 992, 990,
    988] and ending [30, 17, 9]; Karras 2 -> [995, 877, 9]; shift-5 linspace 35 -> [999, 993, 987, ...,
    232, 128]. Bit-exact.
  * numpy's RandomState(0).standard_normal published values (misc.py:158-179 uses it). Bit-exact.
  * tests/golden/*.json (tests/golden/make_golden.py): regression pins of the oracle itself.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.sampler import arch_invariant_rand, frame_mask
from oracle.unipc import UniPC, schedule

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_schedule_matches_reference_recorded_values():
    ts, sg = schedule(35, 5.0, use_karras=True)
    assert len(ts) == 36 and ts.dtype == torch.int64 and len(sg) == 37
    assert ts[:6].tolist() == [995, 994, 993, 992, 990, 988]
    assert ts[-3:].tolist() == [30, 17, 9]
    assert schedule(2, 5.0, use_karras=True)[0].tolist() == [995, 877, 9]
    ts5, sg5 = schedule(35, 5.0, use_karras=False)
    assert len(ts5) == 35 and ts5[:3].tolist() == [999, 993, 987] and ts5[-2:].tolist() == [232, 128]
    assert sg5[-1].item() == 0.0 and sg5.dtype == torch.float32


def test_schedules_golden():
    gold = json.load(open(os.path.join(GOLD, "schedules.json")))
    for name, (n, karras) in {"karras35": (35, True), "karras2": (2, True), "shift5_35": (35, False)}.items():
        ts, sg = schedule(n, 5.0, karras)
        assert ts.tolist() == gold[name]["timesteps"]
        assert sg.tolist() == gold[name]["sigmas"]


def test_noise_matches_numpy_published_values():
    # np.random.RandomState(0).standard_normal: 1.76405235, 0.40015721, 0.97873798, 2.2408932, 1.86755799
    n = arch_invariant_rand((1, 16, 2, 4, 4), 0).flatten()
    ref = np.array([1.76405235, 0.40015721, 0.97873798, 2.2408932, 1.86755799], dtype=np.float32)
    assert np.allclose(n[:5].numpy(), ref, atol=1e-7)
    gold = json.load(open(os.path.join(GOLD, "noise.json")))
    assert n[:8].tolist() == gold["first8"]


def test_unipc_trajectory_golden():
    gold = json.load(open(os.path.join(GOLD, "unipc_traj.json")))
    u = UniPC(3, shift=5.0, use_karras=False)
    x = torch.linspace(-1.5, 1.5, 8)
    for i, t in enumerate(u.timesteps):
        x = u.step(torch.sin(x * 2.0 + i), t, x)
        assert x.tolist() == gold["trajectory"][i]


def test_unipc_orders_and_warmup():
    """Order warm-up (1 then 2) and lower_order_final (last step order 1), fm_solvers_unipc.py:689-694."""
    u = UniPC(4, shift=5.0)
    x = torch.zeros(4)
    orders = []
    for t in u.timesteps:
        x = u.step(torch.ones(4), t, x)
        orders.append(u.this_order)
    assert orders == [1, 2, 2, 1]


def test_unipc_exact_for_linear_flow():
    """With the exact velocity of a straight rectified-flow path, every x0 prediction is the target
    and the sampler lands on it (a property the reference's solver has by construction)."""
    target = torch.tensor([0.3, -1.2, 2.0])
    noise = torch.tensor([1.0, 0.5, -0.7])
    u = UniPC(10, shift=5.0)
    s0 = u.sigmas[0]
    x = (1 - s0) * target + s0 * noise  # start on the straight path x_s = (1-s) x0 + s eps
    for t in u.timesteps:
        x = u.step(noise - target, t, x)
    assert torch.allclose(x, target, atol=1e-5)


def test_frame_mask_rules():
    m = frame_mask(1, 5, 2, 2, 2)
    assert m[0, 0, :, 0, 0].tolist() == [1, 1, 0, 0, 0]
    assert frame_mask(1, 1, 2, 2, 1).sum() == 0  # image batch: no conditioning frames
