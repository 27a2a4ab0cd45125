"""The self-attention's phase anatomy INSIDE the DiT (lab probe build, tools/lab/build.sh probe -DCP25_ATTN_PROBE):
one sampler evaluation of the metric geometry with unit q/k norm weights (zero-shift loop) and one with norm weights
uniform in [0.5, 3] (online max), probe stamps of the evaluation's last self-attention launch (block 27): cycles per
tile, in-kernel clock, and (online form) how many tiles moved a row's shift. Explains the in-bench cost of trained-size
weights against the isolated kernel (tools/bench_attn.py). usage: python tools/probe_in_dit.py [--t0 800]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cosmos_predict2 import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--t0", type=int, default=800)
    ap.add_argument("--wg", type=int, default=64)
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "lab", "libcp25_probe.so"))
    a = ap.parse_args()
    N._LIB_PATH = a.lib
    from bench_attn import probe_report
    from cosmos_predict2.pipeline import DEFAULT_NEGATIVE_PROMPT, Video2WorldInference

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lib = N.load_library()
    lib.cp25_attn_probe_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    h, w, state_t = 704, 1280, 31
    pipe = Video2WorldInference("2B/post-trained", context_parallel_size=1, device=dev, state_t=state_t)
    model = pipe.model
    net = model.net
    frames = model.tokenizer.get_pixel_num_frames(state_t)
    rng = np.random.RandomState(3)
    vid = torch.zeros(1, 3, frames, h, w, dtype=torch.uint8)
    vid[0, :, 0] = torch.from_numpy(rng.randint(0, 256, size=(3, h, w), dtype=np.uint8))
    batch = pipe._get_data_batch_input(vid, "A robot arm pours coffee into a mug on a kitchen counter.", 1,
                                       DEFAULT_NEGATIVE_PROMPT)
    state_shape = (model.config.state_ch, state_t, h // 8, w // 8)
    buf = torch.zeros(a.wg * 8 * (32 * 4 + 8), dtype=torch.int64, device=dev)
    names = [k for k in net.sd if k.endswith(("q_norm.weight", "k_norm.weight"))]
    gw = torch.Generator(device=dev).manual_seed(7)
    w_tr = {k: (0.5 + 2.5 * torch.rand(net.sd[k].shape, device=dev, generator=gw)).to(net.sd[k].dtype) for k in names}
    out = {}
    with torch.no_grad():
        gt = model.encode_conditioning(batch["video"], 1, state_t)
        for tag in ("unit", "trained"):
            if tag == "trained":
                for k in names:
                    net.sd[k].copy_(w_tr[k])
                net.refresh_norm_bounds()
            run = model.begin_sampling(gt, batch["t5_text_embeddings"], batch["neg_t5_text_embeddings"],
                                       state_shape=state_shape, num_conditional_frames=1, guidance=7, seed=0,
                                       num_steps=35)
            run.step()
            torch.cuda.synchronize()
            lib.cp25_attn_probe_set(ctypes.c_void_p(buf.data_ptr()), a.t0, a.wg)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run.step()
            e1.record()
            torch.cuda.synchronize()
            lib.cp25_attn_probe_set(None, 0, 0)
            pb = buf.cpu().numpy()
            n_t = a.wg * 8 * 128
            r = probe_report(pb[:n_t].reshape(a.wg, 8, 32, 4), pb[n_t:].reshape(a.wg, 8, 8))
            r["eval_ms_probe_build"] = e0.elapsed_time(e1)
            r["attention_kernels"] = net.attention_kernels(state_t * (h // 16) * (w // 16))
            out[tag] = r
            print(tag, json.dumps(r), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
