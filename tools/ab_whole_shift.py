"""(Written before long-key launches took the fixed shift up to a bound product of 110: since then the inflated q bound
below no longer selects the zero shift, so the unit-weight A/B compares the fixed shift with itself; the --trained
A/B is unaffected. Results: profiles/r6/shift_power/.)
A/B of the self-attention's softmax-shift form inside the metric's sampler evaluation (round 6): the whole-bound
fixed shift (the default for bound products <= 63: each row shifted by floor(|q_row| max|k|), P <= 2) vs the zero
shift (forced by inflating every block's q bound so the product lands at 80, inside the zero-shift window), evaluation
by evaluation in one process, in ABBA order so that clock drift over the run cancels. The bench.py workload
(Predict2.5-2B Image2World 704x1280x121f, CFG 2, B = 2, L = 109 120, unit norm weights).

  python tools/ab_whole_shift.py [--pairs 6] [--trained]
--trained: q/k norm weights uniform in [0.5, 3] (bound product ~147: the online max) and the A/B is the gated pair
(net.data_tight_k_bound: blocks whose measured bound is <= 110 run the fixed shift on it) against the online max.
Prints one JSON line: ms per evaluation for each form (list and median), their ratio and the kernel names.
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
    ap.add_argument("--trained", action="store_true")
    a = ap.parse_args()
    from cosmos_predict2 import _native as N
    from cosmos_predict2.pipeline import DEFAULT_NEGATIVE_PROMPT, Video2WorldInference

    dev = torch.device("cuda:0")
    N.load_library()
    h, w, state_t = 704, 1280, 31
    pipe = Video2WorldInference("2B/post-trained", context_parallel_size=1, device=dev, state_t=state_t)
    model = pipe.model
    net = model.net
    L = state_t * (h // 16) * (w // 16)
    if a.trained:
        gw = torch.Generator(device=dev).manual_seed(7)
        for k_, w_ in net.sd.items():
            if k_.endswith(("q_norm.weight", "k_norm.weight")):
                w_.copy_((0.5 + 2.5 * torch.rand(w_.shape, device=dev, generator=gw)).to(w_.dtype))
        net.refresh_norm_bounds()
    whole = list(net.attn_bounds)
    c = 128 ** -0.5 * 1.4426950408889634
    zero = [(80.0 / (c * kb), kb) if qb * c * kb < 80.0 else (qb, kb) for qb, kb in whole]
    frames = model.tokenizer.get_pixel_num_frames(state_t)
    rng = np.random.RandomState(3)
    vid = torch.zeros(1, 3, frames, h, w, dtype=torch.uint8)
    vid[0, :, 0] = torch.from_numpy(rng.randint(0, 256, size=(3, h, w), dtype=np.uint8))
    batch = pipe._get_data_batch_input(vid, "A robot arm pours coffee into a mug on a kitchen counter.", 1,
                                       DEFAULT_NEGATIVE_PROMPT)
    st = (model.config.state_ch, state_t, h // 8, w // 8)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    names = {}
    with torch.no_grad():
        gt = model.encode_conditioning(batch["video"], 1, state_t)
        run = model.begin_sampling(gt, batch["t5_text_embeddings"], batch["neg_t5_text_embeddings"], state_shape=st,
                                   num_conditional_frames=1, guidance=7, seed=0, num_steps=35)

        def one(form):
            if a.trained:  # "whole": the gated pair (fixed shift on the measured key bound), "zero": the online max
                net.data_tight_k_bound = form == "whole"
            else:
                net.attn_bounds = whole if form == "whole" else zero
            names[form] = net.attention_kernels(L)["self"]
            if run.done:
                run.restart()
            torch.cuda.synchronize()
            ev0.record()
            run.step()
            ev1.record()
            torch.cuda.synchronize()
            return ev0.elapsed_time(ev1)

        for f in ("whole", "zero", "whole", "zero"):  # warm both
            one(f)
        t = {"whole": [], "zero": []}
        for i in range(a.pairs):
            order = ("whole", "zero") if i % 2 == 0 else ("zero", "whole")
            for f in order:
                t[f].append(round(one(f), 2))
        net.attn_bounds = whole
        net.data_tight_k_bound = False
    med = {f: float(np.median(v)) for f, v in t.items()}
    print(json.dumps({"ms_per_eval": t, "median": med, "whole_over_zero": med["whole"] / med["zero"],
                      "kernels": names, "trained_norm_weights": a.trained}))


if __name__ == "__main__":
    main()
