"""A/B of the self-attention kernel forms inside the metric's sampler evaluation (round 6): attn_fwd_m16 vs attn_fwd_w64
(cp25_attn_self_select 0 / 2), evaluation by evaluation in one process, in ABBA order so that clock drift over the run
cancels. The bench.py workload (Predict2.5-2B Image2World 704x1280x121f, CFG 2, B = 2, L = 109 120).

  python tools/ab_self_form.py [--pairs 6] [--norm-weights lo,hi]
Prints one JSON line: ms per evaluation for each form (list and median) and their ratio.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=6)
    ap.add_argument("--norm-weights", default="", help="lo,hi: q/k norm weights uniform in [lo, hi] (online max)")
    a = ap.parse_args()
    from cosmos_predict2 import _native as N
    from cosmos_predict2.pipeline import DEFAULT_NEGATIVE_PROMPT, Video2WorldInference

    dev = torch.device("cuda:0")
    N.load_library()
    h, w, state_t = 704, 1280, 31
    pipe = Video2WorldInference("2B/post-trained", context_parallel_size=1, device=dev, state_t=state_t)
    model = pipe.model
    if a.norm_weights:
        lo, hi = (float(x) for x in a.norm_weights.split(","))
        gw = torch.Generator(device=dev).manual_seed(7)
        for k_, w_ in model.net.sd.items():
            if k_.endswith(("q_norm.weight", "k_norm.weight")):
                w_.copy_((lo + (hi - lo) * torch.rand(w_.shape, device=dev, generator=gw)).to(w_.dtype))
        model.net.refresh_norm_bounds()
    frames = model.tokenizer.get_pixel_num_frames(state_t)
    rng = np.random.RandomState(3)
    vid = torch.zeros(1, 3, frames, h, w, dtype=torch.uint8)
    vid[0, :, 0] = torch.from_numpy(rng.randint(0, 256, size=(3, h, w), dtype=np.uint8))
    batch = pipe._get_data_batch_input(vid, "A robot arm pours coffee into a mug on a kitchen counter.", 1,
                                       DEFAULT_NEGATIVE_PROMPT)
    st = (model.config.state_ch, state_t, h // 8, w // 8)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        gt = model.encode_conditioning(batch["video"], 1, state_t)
        run = model.begin_sampling(gt, batch["t5_text_embeddings"], batch["neg_t5_text_embeddings"], state_shape=st,
                                   num_conditional_frames=1, guidance=7, seed=0, num_steps=35)

        def one(form):
            N.attn_self_select(form)
            if run.done:
                run.restart()
            torch.cuda.synchronize()
            ev0.record()
            run.step()
            ev1.record()
            torch.cuda.synchronize()
            return ev0.elapsed_time(ev1)

        for f in (0, 2, 0, 2):  # warm both
            one(f)
        t = {0: [], 2: []}
        for i in range(a.pairs):
            order = (0, 2) if i % 2 == 0 else (2, 0)
            for f in order:
                t[f].append(round(one(f), 2))
        N.attn_self_select(1)
    med = {f: float(np.median(v)) for f, v in t.items()}
    print(json.dumps({"m16_ms_per_eval": t[0], "w64_ms_per_eval": t[2], "m16_median": med[0], "w64_median": med[2],
                      "w64_over_m16": med[2] / med[0], "norm_weights": a.norm_weights or "ones (init)",
                      "kernels": model.net.attention_kernels(state_t * (h // 16) * (w // 16))}))


if __name__ == "__main__":
    main()
