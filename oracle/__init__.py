"""CPU oracle for the cosmos-predict2.5 sampler hot path — TEST INFRASTRUCTURE ONLY.

A restatement, in plain PyTorch-CPU / numpy, of the reference's arithmetic for the hot path
(UniPC schedule + update, numpy noise, V2W conditioning, the MiniTrainDIT/MinimalV1LVGDiT forward,
the Wan2.1 VAE), written from the reference files read as text; every function cites the
reference file:line it follows (paths relative to the reference repository root).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and
only as the checker / CPU baseline. The product (cosmos-predict2.5_amd/cosmos_predict2) never
imports it and has no CPU fallback.

Pinning (see DESIGN.md "Oracle"):
  * schedule (unipc.py): pinned to the reference's own outputs recorded in SURVEY.md F3
    (Karras 35 -> [995, 994, 993, 992, 990, 988, ..., 30, 17, 9], Karras 2 -> [995, 877, 9],
    shift-5 linspace -> [999, 993, 987, ..., 232, 128]); tests/golden/schedules.json.
  * noise (noise.py): numpy RandomState(seed).standard_normal — pinned by numpy's published
    values for seed 0.
  * DiT / VAE / attention: "parity unpinned" — the reference's numerics live in third-party
    kernels (transformer-engine RMSNorm/RoPE, flash-attn/cuDNN SDPA, cuDNN conv) and executing the
    reference's network code here was refused; the restatement follows the
    reference source and the standard formulas of those kernels.
"""
