"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

  python tests/golden/make_golden.py

schedules.json   : UniPC timesteps/sigmas (Karras 35, Karras 2, shift-5 35). The timesteps are the
                   values the reference's own FlowUniPCMultistepScheduler produced:
                   tests/test_oracle_golden.py pins them to those recorded values.
unipc_traj.json  : a 3-step UniPC trajectory on a fixed 8-element input with a fixed fake velocity.
noise.json       : arch_invariant_rand((1,16,2,4,4), seed=0) first 8 values (numpy RandomState).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import torch  # noqa: E402

from oracle.sampler import arch_invariant_rand  # noqa: E402
from oracle.unipc import UniPC, schedule  # noqa: E402


def main():
    sch = {}
    for name, (n, karras) in {"karras35": (35, True), "karras2": (2, True), "shift5_35": (35, False)}.items():
        ts, sg = schedule(n, 5.0, karras)
        sch[name] = {"timesteps": ts.tolist(), "sigmas": [float(x) for x in sg.tolist()]}
    json.dump(sch, open(os.path.join(HERE, "schedules.json"), "w"), indent=1)

    u = UniPC(3, shift=5.0, use_karras=False)
    x = torch.linspace(-1.5, 1.5, 8)
    traj = []
    for i, t in enumerate(u.timesteps):
        v = torch.sin(x * 2.0 + i)
        x = u.step(v, t, x)
        traj.append([float(a) for a in x.tolist()])
    json.dump({"x0": torch.linspace(-1.5, 1.5, 8).tolist(), "velocity": "sin(2 x + i)", "trajectory": traj},
              open(os.path.join(HERE, "unipc_traj.json"), "w"), indent=1)

    n = arch_invariant_rand((1, 16, 2, 4, 4), 0).flatten()[:8]
    json.dump({"seed": 0, "shape": [1, 16, 2, 4, 4], "first8": [float(a) for a in n.tolist()]},
              open(os.path.join(HERE, "noise.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
