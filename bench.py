"""Benchmark: frames/sec of Predict2.5-2B Image2World at 704x1280 x 121 frames, 35 UniPC steps.

The workload is one Image2World video through the product model (Video2WorldModelRectifiedFlow):
VAE encode of the conditioning frame, sampler setup (noise, schedule, per-prompt text context),
35 Karras UniPC steps = 36 sampler evaluations, VAE decode of all 31 latent frames to 121 frames.

One bench *step* = one full-geometry sampler evaluation (SamplingRun.step(): patchify + frame
replacement, the CFG-batched B = 2 DiT forward on the 2B net at latent [16, 31, 88, 160],
L = 109 120 tokens, GT-frame velocity replacement + CFG, fused UniPC update). The encode, the setup
and the 121-frame decode are timed once each in the same run (barrier + synchronize around each);
  modeled = frames / (t_encode + t_setup + evals_per_video * t_step + t_decode)
and, by default, one whole video is then timed end to end (encode + every evaluation + decode, barrier +
synchronize around it): value = frames / t_whole_video (--no-whole-video: value = the modeled figure).
Synthetic data: seeded random weights with the 2B shapes, a random conditioning image, N(0, 1) text
embeddings [1, 512, 100352]. bf16 compute.

  python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 (one rank per GPU, RCCL; under torch.distributed.run, or started by bench.py itself when launched plainly): the video's token sequence is sharded context-parallel over
the N ranks (K/V all-gather over xGMI), the decode is banded over the ranks; all ranks work on the
same video (strong scaling). Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cosmos-predict2.5_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "frames/sec, Predict2.5-2B Image2World 720p×121f, 35 UniPC steps, CP=1/8"
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA
HIPBLASLT_BEST_BF16_TFLOPS = 1499.4  # measured: hipBLASLt bf16 16384^3, random data (profiles/r2/peak/peak_gemm.log)
# measured: register-only v_mfma_f32_16x16x32_bf16 loop on random data, no memory traffic at all (the shape the
# self-attention kernel runs; tools/lab/mfma_power.hip, profiles/r2/attn_m16/mfma_power_16x16x32.log)
MFMA_LOOP_BF16_TFLOPS = 1880.3
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r6", "bench_pmc", "pmc_self.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed sampler evaluations")
    ap.add_argument("--warmup", type=int, default=2, help="untimed sampler evaluations before timing")
    ap.add_argument("--num-steps", type=int, default=35, help="UniPC steps (35 = the metric)")
    ap.add_argument("--frames", type=int, default=121)
    ap.add_argument("--model", default="2B/post-trained",
                    help="2B/post-trained: Karras, 36 evals (the metric); 2B/pre-trained: shift-5 linspace, 35 evals "
                         "(SURVEY.md 8(d)'s second variant)")
    ap.add_argument("--resolution", default="704,1280")
    ap.add_argument("--linear-precision", default="bf16", choices=("bf16", "fp8"),
                    help="fp8: the DiT block projections/MLP as fp8 MFMA GEMMs (config 5's option; not the metric)")
    ap.add_argument("--attention-precision", default="bf16", choices=("bf16", "fp8qk", "fp8"),
                    help="fp8qk: self-attention Q K^T on e4m3 operands; fp8: also P.V on e5m2 P / e4m3 V (config 5's "
                         "option; not the metric)")
    ap.add_argument("--norm-weights", default="",
                    help="lo,hi: every q/k RMSNorm weight uniform in [lo, hi] (seeded) instead of the init's ones -- the "
                         "attention then runs the form a trained checkpoint gets (the report names it)")
    ap.add_argument("--no-data-tight-k-bound", action="store_true",
                    help="trained-size norm weights: the online max instead of the gated pair on the measured key "
                         "bound (dit.data_tight_k_bound, on by default since round 6)")
    ap.add_argument("--no-whole-video", action="store_true",
                    help="skip the end-to-end video (value is then the per-evaluation model; for quick A/B runs)")
    ap.add_argument("--no-cfg-share", action="store_true",
                    help="every CFG entry computes block 0's shared self-attention prefix (A/B of the sharing)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: the host cores this process may use, capped by OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu-config1", action="store_true",
                    help="skip the CPU leg's end-to-end BASELINE config 1 video (~30-60 s with the weight setup; on by "
                         "default: the whole-video CPU baseline SURVEY.md §8(d) asks for)")
    ap.add_argument("--trained-evals", type=int, default=4,
                    help="N = 1: after the metric run, time this many evaluations with q/k norm weights uniform in "
                         "[0.5, 3] (the attention form a trained checkpoint gets) as the line's trained_norm_weights "
                         "sub-record (0: skip)")
    ap.add_argument("--backend", default="nccl", help="process-group backend for N > 1 (nccl = RCCL; gloo only "
                    "for rehearsing the multi-rank flow with several ranks on one GPU, see --share-device)")
    ap.add_argument("--share-device", action="store_true", help="every rank uses cuda:0 (rehearsal on one GPU)")
    return ap.parse_args()


def _heartbeat(rank: int, period: float = 30.0) -> None:
    """Progress line on stderr every `period` s (keeps watchdogs informed)."""
    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            print(f"[bench rank {rank}] running {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


class _Timer:
    """Barrier + device synchronize on both sides; max over ranks."""

    def __init__(self, world: int, dev):
        self.world, self.dev = world, dev

    def _sync(self):
        torch.cuda.synchronize(self.dev)
        if self.world > 1:
            dist.barrier()

    def __call__(self, fn):
        self._sync()
        t0 = time.perf_counter()
        out = fn()
        self._sync()
        el = time.perf_counter() - t0
        if self.world > 1:
            tt = torch.tensor([el], device=self.dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = tt.item()
        return out, el


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start the N ranks as one torch.distributed.run child (one
    process per GPU, LOCAL_RANK = GPU index, rendezvous on 127.0.0.1, the reference's torchrun ->
    examples/inference.py flow) and return its exit code. Called before anything touches the GPU; the parent
    never execs."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        raise SystemExit(launch_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    if a.steps < 1:
        raise SystemExit("--steps must be >= 1")
    _heartbeat(rank)
    dev = torch.device("cuda", 0 if a.share_device else local)
    torch.cuda.set_device(dev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(a.backend)

    from cosmos_predict2.pipeline import DEFAULT_NEGATIVE_PROMPT, Video2WorldInference
    from cosmos_predict2 import _native

    _native.load_library()
    h, w = (int(x) for x in a.resolution.split(","))
    state_t = 1 + (a.frames - 1) // 4
    pipe = Video2WorldInference(a.model, context_parallel_size=world, device=dev, state_t=state_t,
                                linear_precision=a.linear_precision, attention_precision=a.attention_precision)
    model = pipe.model
    model.net.share_cfg_block0 = not a.no_cfg_share
    model.net.data_tight_k_bound = not a.no_data_tight_k_bound
    if a.norm_weights:
        lo, hi = (float(x) for x in a.norm_weights.split(","))
        gw = torch.Generator(device=dev).manual_seed(7)
        for k_, w_ in model.net.sd.items():
            if k_.endswith(("q_norm.weight", "k_norm.weight")):
                w_.copy_((lo + (hi - lo) * torch.rand(w_.shape, device=dev, generator=gw)).to(w_.dtype))
        model.net.refresh_norm_bounds()
    karras = model.config.use_kerras_sigma_at_inference
    frames = model.tokenizer.get_pixel_num_frames(state_t)
    # conditioning "image": frame 0 random uint8, later frames zero (read_and_process_image layout)
    rng = np.random.RandomState(3)
    vid = torch.zeros(1, 3, frames, h, w, dtype=torch.uint8)
    vid[0, :, 0] = torch.from_numpy(rng.randint(0, 256, size=(3, h, w), dtype=np.uint8))
    batch = pipe._get_data_batch_input(vid, "A robot arm pours coffee into a mug on a kitchen counter.", 1,
                                       DEFAULT_NEGATIVE_PROMPT)
    state_shape = (model.config.state_ch, state_t, h // 8, w // 8)
    timer = _Timer(world, dev)

    # ---- kernel-load prime (untimed): encode, one evaluation, a 2-latent-frame decode
    with torch.no_grad():
        gt = model.encode_conditioning(batch["video"], 1, state_t)
        run = model.begin_sampling(gt, batch["t5_text_embeddings"], batch["neg_t5_text_embeddings"],
                                   state_shape=state_shape, num_conditional_frames=1, guidance=7, seed=0,
                                   num_steps=a.num_steps)
        run.step()
        model.decode(run.latents()[:, :, :2])
        del run, gt

        # ---- per-video pieces timed once
        gt, t_enc = timer(lambda: model.encode_conditioning(batch["video"], 1, state_t))
        run, t_setup = timer(lambda: model.begin_sampling(
            gt, batch["t5_text_embeddings"], batch["neg_t5_text_embeddings"], state_shape=state_shape,
            num_conditional_frames=1, guidance=7, seed=0, num_steps=a.num_steps))
        evals = run.num_evals

        def advance(k):
            for _ in range(k):
                if run.done:  # more evaluations than one trajectory: start it over (same work per step)
                    run.restart()
                run.step()

        advance(a.warmup)
        net = model.net
        net.attn_events = []
        net.comm_events = [] if world > 1 else None
        _, t_steps = timer(lambda: advance(a.steps))
        ev = net.attn_events
        cev = net.comm_events
        net.attn_events = net.comm_events = None
        t_step = t_steps / a.steps
        lat = run.latents()
        video, t_dec = timer(lambda: model.decode(lat))
        assert video.shape[2] == frames and torch.isfinite(video.float()).all()
        del video
        t_whole = None
        if not a.no_whole_video:
            def whole():
                g0 = model.encode_conditioning(batch["video"], 1, state_t)
                r0 = model.begin_sampling(g0, batch["t5_text_embeddings"], batch["neg_t5_text_embeddings"],
                                          state_shape=state_shape, num_conditional_frames=1, guidance=7, seed=0,
                                          num_steps=a.num_steps)
                while not r0.done:
                    r0.step()
                return model.decode(r0.latents())

            vid_w, t_whole = timer(whole)
            assert torch.isfinite(vid_w.float()).all()
            del vid_w

        # ---- trained-size q/k norm weights (a modelled sub-record): the attention takes the form a real checkpoint
        # gets (online max; the synthetic unit weights give the zero-shift loop). Same geometry, a second sampling run
        # (its per-prompt cross-attention K/V are normed with the trained-size weights); unit-weight and trained-weight
        # evaluations alternate, one each per pair, so clock drift over the run cannot bias the ratio
        kernels_metric = net.attention_kernels(state_t * (h // 16) * (w // 16))  # before the weights change below
        trained = None
        if world == 1 and not a.norm_weights and a.trained_evals > 0:
            names = [k_ for k_ in net.sd if k_.endswith(("q_norm.weight", "k_norm.weight"))]
            w_unit = {k_: net.sd[k_].clone() for k_ in names}
            gw = torch.Generator(device=dev).manual_seed(7)
            w_tr = {k_: (0.5 + 2.5 * torch.rand(net.sd[k_].shape, device=dev, generator=gw)).to(net.sd[k_].dtype)
                    for k_ in names}

            def use(ws):
                for k_ in names:
                    net.sd[k_].copy_(ws[k_])
                net.refresh_norm_bounds()

            use(w_tr)
            run_t = model.begin_sampling(gt, batch["t5_text_embeddings"], batch["neg_t5_text_embeddings"],
                                         state_shape=state_shape, num_conditional_frames=1, guidance=7, seed=0,
                                         num_steps=a.num_steps)
            run_t.step()  # warm (the online-max kernel's first launch)
            kernels_tr = net.attention_kernels(state_t * (h // 16) * (w // 16))

            def step_t():
                if run_t.done:
                    run_t.restart()
                run_t.step()

            t_u, t_t, ms_tr = [], [], []
            for _ in range(a.trained_evals):
                use(w_unit)
                t_u.append(timer(lambda: advance(1))[1])
                use(w_tr)
                net.attn_events = []
                t_t.append(timer(step_t)[1])
                fl = max((f for _, _, f in net.attn_events), default=0.0)
                ms_tr += [e0.elapsed_time(e1) for e0, e1, f in net.attn_events if f == fl]
                net.attn_events = None
            use(w_unit)
            t_tr = sum(t_t) / len(t_t)
            trained = {
                "norm_weights": "q/k RMSNorm weights uniform in [0.5, 3] (seeded; bound product ~147 > 96)",
                "evals_timed": a.trained_evals,
                "ms_per_eval": t_tr * 1e3,
                "unit_weights_ms_per_eval_interleaved": sum(t_u) / len(t_u) * 1e3,
                "vs_unit_weights_ms_per_eval": t_tr / (sum(t_u) / len(t_u)),
                "modeled_value": frames / (t_enc + t_setup + evals * t_tr + t_dec),
                "value_method": "per-evaluation model with this run's encode, setup and decode times; the unit- and "
                                "trained-weight evaluations alternate in one process",
                "self_attention_avg_launch_ms": sum(ms_tr) / len(ms_tr) if ms_tr else None,
                "attention_kernels": kernels_tr,
            }

    video_s = t_enc + t_setup + evals * t_step + t_dec
    # dominant kernel: self-attention flash kernel, HIP events on its launch stream around every
    # launch in the timed steps
    # launch; the CFG pair's shared block-0 self-attention (B = 1, half the FLOP) is left out of the average
    attn_flop = max((f for _, _, f in ev), default=0.0)
    attn_ms = [e0.elapsed_time(e1) for e0, e1, f in ev if f == attn_flop]
    n_shared = sum(1 for _, _, f in ev if f != attn_flop)
    attn_avg_s = (sum(attn_ms) / len(attn_ms)) / 1e3 if attn_ms else float("nan")
    achieved = attn_flop / attn_avg_s / 1e12 if attn_ms else 0.0

    # context parallel: per rank, the exposed K/V gather waits (HIP events on the compute stream around each wait) and
    # the self-attention launches of the timed steps, per evaluation
    cp_report = None
    if world > 1:
        mine = {"rank": rank, "gather_wait_ms_per_eval": sum(e0.elapsed_time(e1) for e0, e1 in cev) / a.steps,
                "gather_waits_per_eval": len(cev) / a.steps,
                "attention_ms_per_eval": sum(e0.elapsed_time(e1) for e0, e1, _ in ev) / a.steps,
                "eval_ms": t_step * 1e3}
        every = [None] * world
        dist.all_gather_object(every, mine)
        cp_report = {"per_rank": every,
                     "max_gather_wait_ms_per_eval": max(r["gather_wait_ms_per_eval"] for r in every),
                     "max_attention_ms_per_eval": max(r["attention_ms_per_eval"] for r in every)}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle.cpu_baseline import config1_end_to_end, dit_block_sample, host_threads

        threads, visible = host_threads(a.cpu_threads or None)
        cpu = dit_block_sample(L=state_t * (h // 16) * (w // 16), threads=threads, forwards=2 * evals, frames=frames)
        cpu["host_cores_visible"] = visible
        if not a.no_cpu_config1:
            cpu["config1_end_to_end"] = config1_end_to_end(threads=threads)
        cpu["cores_note"] = (f"{threads} of {visible} host threads: the GPU box's CPU share for a one-GPU job is 16 "
                             "(OMP_NUM_THREADS=16 there); its affinity mask lists every core of the shared host")

    if rank == 0:
        valid = (a.num_steps == 35 and a.frames == 121 and (h, w) == (704, 1280) and a.model == "2B/post-trained"
                 and a.linear_precision == "bf16" and a.attention_precision == "bf16" and not a.norm_weights)
        # HBM bytes per self-attention launch: a static prior from the committed rocprofv3 PMC passes of
        # this kernel at this shape (tools/pmc_attn.sh; FETCH_SIZE x2 gfx950 correction + WRITE_SIZE),
        # not collected in this run; only the CP = 1 metric shape was measured, other shapes report null
        traffic, traffic_src = None, None
        if world == 1 and valid and os.path.exists(PMC_SUMMARY):
            with open(PMC_SUMMARY) as f:
                traffic = json.load(f).get("traffic_bytes_per_launch")
            traffic_src = "static prior: " + os.path.relpath(PMC_SUMMARY, ROOT) + " (rocprofv3 PMC, not this run)"
        modeled = frames / video_s
        line = {
            "metric": METRIC,
            "value": frames / t_whole if t_whole is not None else modeled,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": t_step * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16" if (a.linear_precision, a.attention_precision) == ("bf16", "bf16") else
                     " + ".join(x for x, on in (("fp8 (block GEMMs)", a.linear_precision == "fp8"),
                                                ("fp8 (attention Q K^T)", a.attention_precision == "fp8qk"),
                                                ("fp8 (attention Q K^T, P.V)", a.attention_precision == "fp8")) if on)
                     + " + bf16",
            "data": "synthetic: seeded random 2B/VAE weights, random conditioning image, N(0,1) text embeddings"
                    + (f", q/k norm weights uniform in [{a.norm_weights}]" if a.norm_weights else ""),
            "value_method": ("whole video timed end to end in this run (encode + every evaluation + decode)"
                             if t_whole is not None else
                             "per-evaluation model: frames / (encode + setup + evals x mean timed evaluation + decode), "
                             "each part timed in this run"),
            "whole_video": None if t_whole is None else {"seconds": t_whole, "frames_per_s": frames / t_whole},
            "modeled_value": modeled,
            "config": {
                "workload": f"Predict2.5-2B Image2World {h}x{w}x{frames}f ({a.model}), {a.num_steps} "
                            + (f"Karras UniPC steps ({evals} evals" if karras else f"shift-5 UniPC steps ({evals} evals")
                            + f" x CFG 2, batched), VAE encode cond frame + decode {frames}f",
                "step": "one sampler evaluation: CFG-batched (B=2) DiT forward + CFG + UniPC update",
                "evals_per_video": evals,
                "seconds_per_video": video_s,
                "encode_s": t_enc,
                "setup_s": t_setup,
                "decode_s": t_dec,
                "latent": [16, state_t, h // 8, w // 8],
                "tokens": state_t * (h // 16) * (w // 16),
                "global_batch": 1,
                "parallelism": f"cp{world}",
                "linear_precision": a.linear_precision,
                "attention_precision": a.attention_precision,
                "cfg_block0_shared": bool(net.share_cfg_block0),
                "norm_weights": a.norm_weights or "ones (init)",
                "attention_kernels": kernels_metric,
                "metric_config": valid,
            },
            "roofline": {
                "bound": "mfma",
                "kernel": {"bf16": "cp25_attn_fwd_prescaled (DiT self-attention, bf16 16x16x32 MFMA, attn_fwd_m16)",
                           "fp8qk": "cp25_attn_fwd_prescaled_fp8qk (DiT self-attention, fp8 Q K^T + bf16 P V MFMA)",
                           "fp8": "cp25_attn_fwd_prescaled_fp8 (DiT self-attention, fp8 Q K^T and P V MFMA)"}[
                               a.attention_precision],
                "achieved": achieved,
                "peak": BF16_DENSE_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / BF16_DENSE_PEAK_TFLOPS,
                # a reference point, not a ceiling: the vendor GEMM's best on this chip with random bf16 data
                # (16384^3, hipBLASLt; power-limited clock, profiles/r2/peak/peak_gemm.log)
                "hipblaslt_best_tflops": HIPBLASLT_BEST_BF16_TFLOPS,
                "frac_of_hipblaslt_best": achieved / HIPBLASLT_BEST_BF16_TFLOPS,
                "mfma_loop_peak": MFMA_LOOP_BF16_TFLOPS,
                "frac_of_mfma_loop": achieved / MFMA_LOOP_BF16_TFLOPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "launches_timed": len(attn_ms),
                "half_launches_excluded": n_shared,
                "avg_launch_ms": attn_avg_s * 1e3,
                "flop_per_launch": attn_flop,
            },
            "cpu_baseline": cpu and {k: cpu[k] for k in ("value", "unit", "cores", "kind", "sample", "host_cores_visible",
                                                         "sample_seconds", "config1_end_to_end", "cores_note") if k in cpu},
        }
        if trained is not None:
            line["trained_norm_weights"] = trained
        if cp_report is not None:
            line["context_parallel"] = cp_report
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
