"""Config 5 geometry on one GPU: action-conditioned autoregressive sliding-window generation
(ActionConditionedInference.generate, the reference's action_conditioned.py:205-380 chunk loop) at the
Bridge resolution 480x640 (action/configs/action_conditioned/data.py:78), 13-frame chunks (12 new
frames each), 35 UniPC steps, CFG 7, synthetic random-init weights, random initial frame and actions.
Reports frames/s of the whole long video; --linear-precision fp8 runs the DiT block GEMMs in fp8; --block-gemm lib puts them on the library (A/B).
One JSON line. (CP = 4 needs four GPUs; this is the single-GPU rate of the same loop.)"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cosmos_predict2.action_conditioned import ActionConditionedInference  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--resolution", default="480,640")
    ap.add_argument("--num-steps", type=int, default=35)
    ap.add_argument("--chunk-size", type=int, default=12)
    ap.add_argument("--linear-precision", default="bf16", choices=("bf16", "fp8"))
    ap.add_argument("--attention-precision", default="bf16", choices=("bf16", "fp8qk", "fp8"))
    ap.add_argument("--hip-graph", action="store_true",
                    help="replay each chunk's DiT forward from a HIP graph after its first evaluation (model.hip_graph)")
    ap.add_argument("--block-gemm", default="own", choices=("own", "lib"),
                    help="block projections on the hand-written GEMMs (default) or the library (A/B)")
    a = ap.parse_args()
    h, w = (int(x) for x in a.resolution.split(","))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n_chunks = -(-(a.frames - 1) // a.chunk_size)
    inf = ActionConditionedInference(device=dev, state_t=1 + a.chunk_size // 4, linear_precision=a.linear_precision,
                                     attention_precision=a.attention_precision)
    if a.block_gemm == "lib":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from library_gemm_net import use_library_gemms
        use_library_gemms(inf.pipe.model.net)
    inf.pipe.model.hip_graph = a.hip_graph
    adim = inf.pipe.model.net.cfg.action_dim
    rng = np.random.RandomState(0)
    img = rng.randint(0, 256, size=(h, w, 3), dtype=np.uint8)
    actions = (rng.standard_normal((n_chunks * a.chunk_size, adim)) * 0.1).astype(np.float32)
    # prime (kernel loads, fp8 weight cache): one chunk at 1 step
    inf.generate(img, actions, chunk_size=a.chunk_size, num_steps=1, single_chunk=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    video = inf.generate(img, actions, chunk_size=a.chunk_size, num_steps=a.num_steps, max_frames=a.frames)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert video.shape == (a.frames, h, w, 3), video.shape
    print(json.dumps({"workload": f"action-conditioned AR {a.frames}f at {h}x{w}, {n_chunks} chunks of "
                                  f"{a.chunk_size + 1} frames, {a.num_steps} UniPC steps, CFG 7",
                      "linear_precision": a.linear_precision, "block_gemm": a.block_gemm, "hip_graph": a.hip_graph,
                      "attention_precision": a.attention_precision, "n_gpus": 1, "seconds": dt,
                      "frames_per_s": a.frames / dt, "s_per_chunk": dt / n_chunks}), flush=True)


if __name__ == "__main__":
    main()
