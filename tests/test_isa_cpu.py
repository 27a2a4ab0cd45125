"""Static ISA checks of the hand-scheduled kernels (CPU: hipcc cross-compiles gfx950 here).

The attention and conv kernels issue LDS reads from inline asm and retire them with counted s_waitcnt lgkmcnt; the
compiler does not know those destinations are written asynchronously. tools/isa_check.py replays each kernel's
instruction stream and fails on any instruction that touches a VGPR while an LDS read into it is in flight (the bug a
dead asm output produced in round 3: the register handed to another value mid-flight, silently wrong row sums). It
also holds the self-attention's MFMA phase free of hazard s_nop pads (the operand-pin form that caused them cost
2.3 %) and of in-loop scratch traffic.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_check  # noqa: E402

CSRC = os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc")
SOURCES = ["attn_fwd.hip", "vae_ops.hip", "vae_attn.hip", "gemm.hip", "gemm_f32.hip"]


@pytest.fixture(scope="module", autouse=True)
def _compile_all():
    """Compile the sources to ISA concurrently once (isa_check caches per source): the checks below then read the
    cache instead of waiting on one hipcc after another."""
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        return
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        list(ex.map(lambda f: isa_check.compile_asm(os.path.join(CSRC, f)), SOURCES))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not installed")
@pytest.mark.parametrize("src", SOURCES)
def test_no_lds_read_races(src):
    rep = isa_check.check(os.path.join(CSRC, src))
    assert rep
    races = {n: r["races"][:2] for n, r in rep.items() if r["races"]}
    assert not races, races


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not installed")
def test_gemm_f32_no_inloop_scratch():
    """cp25_gemm_f32's kernel double-buffers the W chunk in the LDS with one barrier per chunk: besides
    the race check above, no scratch traffic inside its loops."""
    rep = isa_check.check(os.path.join(CSRC, "gemm_f32.hip"))
    assert rep
    bad = {n: r["inloop_scratch"] for n, r in rep.items() if r["inloop_scratch"]}
    assert not bad, bad


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not installed")
def test_attention_m0_only_in_dma_asm():
    """The attention's LDS-DMA asm writes M0 undeclared (reserved: the compiler never allocates it and ignores a
    clobber of it); no compiler-emitted instruction of any attention kernel may name M0."""
    rep = isa_check.check(os.path.join(CSRC, "attn_fwd.hip"))
    assert rep
    bad = {n: r["m0_uses"][:2] for n, r in rep.items() if r["m0_uses"]}
    assert not bad, bad


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not installed")
def test_self_attention_loop_shape():
    rep = isa_check.check(os.path.join(CSRC, "attn_fwd.hip"), "attn_fwd_m16ILi0ELb1ELi1ELb0ELi0ELi0EE")
    (r,) = rep.values()  # the bench's kernel: self-attention, prescaled q, zero shift
    # scratch traffic only in the loop's cold contract-guard branch (a NaN poison of overflowed rows), never in the
    # MFMA / softmax phases: at most the one reload + one spill of the NaN fill
    assert r["inloop_scratch"] <= 2, r["inloop_scratch"]
    # hazard pads inside the tile loop (the MFMA / softmax phases): 12 now, 192 with round 3's operand-redefining wait
    # pins; the whole kernel's count also holds the prologue's q normalisation pads (rsqrt, packed f32), outside the loop
    assert r["inloop_nops"] <= 16, r["inloop_nops"]
    assert r["nops"] <= 64, r["nops"]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not installed")
def test_self_attention_fixed_shift_loop_shape():
    """The fixed-shift instantiation, the bench's kernel since round 6 (the whole-bound shift, m16_mode whole_ok): its
    per-row shift rides as the Q K^T chains' initial C, 8 more live VGPRs at the 256 cap. Its in-loop scratch is
    confined to cold branches (the ragged last key tile's DMA offsets and the contract guard): at most 8 such
    instructions, none in the MFMA / softmax phases' straight-line code; hazard pads as in the zero-shift loop."""
    rep = isa_check.check(os.path.join(CSRC, "attn_fwd.hip"), "attn_fwd_m16ILi0ELb1ELi0ELb0ELi0ELi0EE")
    (r,) = rep.values()
    assert r["inloop_scratch"] <= 8, r["inloop_scratch"]
    assert r["inloop_nops"] <= 16, r["inloop_nops"]
    assert r["nops"] <= 64, r["nops"]


_SYNTH = """_Zk:
\tds_read_b128 v[0:3], v10
\ts_cbranch_scc1 .LBB0_2
\ts_waitcnt lgkmcnt(0)
\ts_branch .LBB0_3
.LBB0_1:
\tv_add_f32_e32 v20, v1, v21
\ts_endpgm
.LBB0_2:
\tv_add_f32_e32 v22, v2, v23
.LBB0_3:
\tv_mov_b32_e32 v3, v24
\ts_endpgm
.Lfunc_end0:
"""


def test_race_check_follows_control_flow():
    """The checker on a hand-made stream: the read of v[0:3] is retired on the fall-through path only, so v2 on the
    branch target is a race and so is v3 where both paths join; the block after the unconditional branch is reached
    by no path with the read in flight (no race there: the checker's linear form reported one)."""
    r = isa_check.analyse(_SYNTH, "_Zk")
    assert r["races"] == ["v_add_f32_e32 v22, v2, v23", "v_mov_b32_e32 v3, v24"]


_SYNTH2 = """_Zm:
\tds_read_b128 v[4:7], v10
\tds_read_b64 a[0:1], v11
\tv_add_f32_e64 v20, -v5, |v21|
\tv_mov_b32_e32 v22, a1
\tds_read_b32 v30, v6 offset:16
\ts_mov_b32 m0, s2
\ts_nop 0
\tglobal_load_lds_dwordx4 v31, s[4:5]
\ts_waitcnt lgkmcnt(0)
\tv_mov_b32_e32 v23, v4
\ts_endpgm
.Lfunc_end1:
"""


def test_race_check_sees_modifiers_agprs_and_addresses():
    """A register behind a source modifier (-v5), an AGPR destination (a1) and a ds_read whose ADDRESS is still in
    flight (v6) are each a race; the s_nop 0 after an M0 write (the LDS-DMA asm's own) is not counted as a hazard pad;
    after lgkmcnt(0) nothing is in flight."""
    r = isa_check.analyse(_SYNTH2, "_Zm")
    assert r["races"] == ["v_add_f32_e64 v20, -v5, |v21|", "v_mov_b32_e32 v22, a1", "ds_read_b32 v30, v6 offset:16"]
    assert r["nops"] == 0 and r["m0_nops"] == 1
