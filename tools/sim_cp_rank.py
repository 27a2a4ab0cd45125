"""Compute cost of one context-parallel rank's DiT forward, simulated on one GPU.

Rank 0 of CP = N at the metric shape (2B, latent [16, 31, 88, 160], L = 109 120, CFG batch 2):
forward_tokens runs exactly as on a real rank (two stream lanes, unsplit attention against all L
keys), except that the RCCL K/V all-gather is replaced by a local copy that fills the gathered
buffer with this rank's shard repeated N times (same bytes written, no xGMI traffic). The measured
time per forward is therefore the rank's compute with zero-cost communication; compare it with
(CP = 1 forward time) / N to see what the lanes cost, and add the exposed all-gather time for a
real N-GPU estimate. Prints one JSON line per N.
usage: python tools/sim_cp_rank.py [--cp 2 4 8] [--iters 2] [--model 14B/pre-trained]
"""
import argparse
import faulthandler
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import torch  # noqa: E402
import torch.distributed  # noqa: E402

from cosmos_predict2 import context_parallel as cpx  # noqa: E402
from cosmos_predict2 import dit as dit_mod  # noqa: E402
from cosmos_predict2.dit import Geometry, MinimalV1LVGDiT, init_state_dict  # noqa: E402
from cosmos_predict2.net_config import MODELS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cp", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--model", default="2B/post-trained", help="net_config.MODELS key (14B: BASELINE config 3)")
    ap.add_argument("--blocks", type=int, default=0, help="0 = the model's own block count")
    ap.add_argument("--geometry", default="31,44,80", help="latent frames, patch rows, patch cols (T,Hp,Wp); "
                    "multi-view: T = views x frames per view")
    ap.add_argument("--views", type=int, default=1, help="views stacked along T (multi-view nets)")
    ap.add_argument("--gather", default="loop", choices=["expand", "loop", "none"],
                    help="how the fake gather fills the buffer: loop = N copies of the shard on the compute stream "
                         "(the copies count as compute time); none = every lane-block reads one persistent buffer "
                         "filled with real gathered K|V rows during the warm-up forward, no copy in the timed ones "
                         "(the rank's compute with communication fully hidden, on realistic data)")
    ap.add_argument("--trace", action="store_true", help="debug: event after every op; on a hang print the "
                    "last completed op of every stream")
    ap.add_argument("--batch1", action="store_true", help="debug: one batch entry (no lanes)")
    ap.add_argument("--no-phase", action="store_true", help="debug: never record lane 0's phase event")
    ap.add_argument("--force-lanes", action="store_true", help="run the two lanes at CP = 1 too")
    ap.add_argument("--lib", default="", help="a lab build of libcp25.so to load instead of the in-tree one (A/B)")
    a = ap.parse_args()
    if a.lib:
        from cosmos_predict2 import _native
        _native._LIB_PATH = a.lib
    faulthandler.dump_traceback_later(90, repeat=True)  # a stuck host shows where
    dev = torch.device("cuda:0")
    cfg = MODELS[a.model][0]
    if a.blocks:
        cfg = cfg.replace(num_blocks=a.blocks)
    T, Hp, Wp = (int(x) for x in a.geometry.split(","))
    if a.views > 1:
        cfg = cfg.replace(state_t=T // a.views)
    net = MinimalV1LVGDiT(cfg, device=dev)
    net.load_state_dict(init_state_dict(cfg, seed=0, device=dev))
    net.force_lanes = a.force_lanes
    L = T * Hp * Wp
    g = torch.Generator(device=dev).manual_seed(0)
    nb = 1 if a.batch1 else 2
    ctx = net.prepare_context(torch.randn(nb, 512 * a.views, cfg.crossattn_proj_in_channels, device=dev,
                                          generator=g).to(torch.bfloat16))
    t_B_T = torch.full((nb, T), 0.877, device=dev)
    state = {"cp": 1, "warm": True, "buf": {}}

    if a.gather == "none":
        def persistent_buffer(shape):  # one buffer per shape, written only in the warm-up forward
            buf = state["buf"].get(tuple(shape))
            if buf is None:
                buf = state["buf"][tuple(shape)] = torch.empty(shape, dtype=torch.bfloat16, device=dev)
            return buf
        net._kv_gather_buffer = persistent_buffer

    def fake_gather(out, x, group):
        n = state["cp"]
        if a.gather == "none":
            if state["warm"]:
                for r in range(n):
                    out.view(n, -1)[r].copy_(x.reshape(-1))
            return cpx._Done()
        if a.gather == "expand":
            out.view(n, -1).copy_(x.reshape(1, -1).expand(n, -1))
        elif a.gather == "loop":
            for r in range(n):
                out.view(n, -1)[r].copy_(x.reshape(-1))
        return cpx._Done()

    dit_mod.all_gather_into_async = fake_gather
    if a.no_phase:
        orig = MinimalV1LVGDiT._cp_self_attention

        def no_phase(self, *args, **kw):
            args = list(args)
            if len(args) >= 11:
                args[10] = None
            kw.pop("phase_event", None)
            return orig(self, *args, **kw)

        MinimalV1LVGDiT._cp_self_attention = no_phase
    torch.distributed.get_world_size = lambda group=None: state["cp"]
    trace = []
    if a.trace:
        from cosmos_predict2 import _native as N
        import torch.nn.functional as F

        def wrap(mod, name):
            fn = getattr(mod, name)

            def w(*args, **kw):
                r = fn(*args, **kw)
                e = torch.cuda.Event()
                e.record()
                trace.append((torch.cuda.current_stream().cuda_stream, name, e))
                return r
            setattr(mod, name, w)
        for nm in ("attn_fwd", "ln_mod", "head_rmsnorm_rope", "copy_rows", "gelu_", "final_ln_mod"):
            wrap(N, nm)
        import types

        dit_mod.F = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("__")})
        wrap(dit_mod.F, "linear")
        wrap(dit_mod, "all_gather_into_async")
    for n in a.cp:
        state["cp"] = n
        net.cp_group = None if n == 1 else object()
        geo = Geometry(T=T, Hp=Hp, Wp=Wp, tok0=0, n_tok=L // n, n_views=a.views)
        rows = torch.randn(geo.n_tok, 1, 72, device=dev, generator=g).to(torch.bfloat16)
        print(f"cp {n}: warm-up forward", flush=True)
        state["warm"] = True
        net.forward_tokens(rows, t_B_T, ctx, geo)  # warm
        state["warm"] = False
        print(f"cp {n}: issued {len(trace)} traced ops", flush=True)
        if a.trace:
            t_end = time.time() + 30
            while time.time() < t_end and not all(e.query() for _, _, e in trace):
                time.sleep(0.5)
            last = {}
            for i, (st, nm, e) in enumerate(trace):
                if e.query():
                    last[st] = (i, nm)
            pending = [(i, st, nm) for i, (st, nm, e) in enumerate(trace) if not e.query()]
            print("last completed per stream:", last, flush=True)
            print("first pending:", pending[:6], flush=True)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            t0 = time.perf_counter()
            net.forward_tokens(rows, t_B_T, ctx, geo)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"model": a.model, "geometry": [T, Hp, Wp], "views": a.views, "cp": n, "gather": a.gather, "blocks": cfg.num_blocks, "tokens_per_rank": geo.n_tok,
                          "forward_s": min(ts), "forward_s_all": ts}), flush=True)


if __name__ == "__main__":
    main()
