"""Lab builds of libcp25.so with a text-patched attn_fwd.hip (isolation variants of the persistent cross-attention's
block boundary, for same-box A/B with tools/bench_xattn.py --lib; results are WRONG for every patch except 'none').
The product source is not touched: the patched copy is compiled from /tmp and linked with the in-tree objects.
usage: python tools/lab/attn_variant.py <name> <patch>[,<patch>...]  ->  tools/lab/libcp25_<name>.so
patches: nostore (no O stores at block boundaries), nodma (no next-block Q copy), noqread (no Q read from LDS),
nostagger (the Q copy at tile 0 in every workgroup; correct results), rowsum_first (correct results),
prio_b_hold, prio_static_b (wave priority forms; correct results), ahead3, ahead4 (operand ring depth;
correct results), hotload, noload (staging-load probes), noexp, noreads (round-5 isolation builds), kv_sc1, kv_nt,
kv_sc0sc1 (the K / V DMA's cache policy, round 6; correct results), none
DEFINES="-D..." adds compile definitions (e.g. -DCP25_ATTN_PROBE for the s_memtime probe)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc")
OBJ = os.path.join(ROOT, "cosmos-predict2.5_amd", "cosmos_predict2", "_lib", "obj")

PATCHES = {
    "nostore": [("      if (row0 + r < a.Lq) *reinterpret_cast<u32x4*>(wo + (int64_t)(row0 + r) * a.o_sl) = v;\n",
                 "      if (row0 + r < 0) *reinterpret_cast<u32x4*>(wo + (int64_t)(row0 + r) * a.o_sl) = v;\n")],
    "nodma": [("      if (t == copy_tile && blk0 + tb + 1 < blk_end) dma_q(blk0 + tb + 1, 0, 8);\n",
               "      if (t == copy_tile && blk0 + tb + 1 < 0) dma_q(blk0 + tb + 1, 0, 8);\n")],
    "noqread": [("      if (t == ntk - 1 && blk0 + tb + 1 < blk_end) {\n",
                 "      if (t == ntk - 1 && blk0 + tb + 1 < 0) {\n")],
    "nostagger": [("constexpr bool kQCopyStagger = true;\n", "constexpr bool kQCopyStagger = false;\n")],  # correct
    # the 4 row-sum MFMAs at the start of the MFMA phase (they need no LDS operand: they cover the first reads' latency)
    # instead of after the P.V pairs; correct results
    "rowsum_first": [("      if constexpr (n == 15) {  // row sums of P(t), after its P.V pairs\n",
                      "      if constexpr (n == 99) {  // row sums of P(t), after its P.V pairs\n"),
                     ("""      static_for<kAhead>(issue);
    }
    static_for<32>([&](auto NC) __attribute__((always_inline)) {""",
                      """      static_for<kAhead>(issue);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb[ks][qh], lsum[qh], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    static_for<32>([&](auto NC) __attribute__((always_inline)) {""")],
    # wave priority: group B (waves 4-7, the later-dispatched half) stays at s_setprio 1 through its softmax phase
    # (A still flips 1 / 0 per phase); or the guide's static form: no per-phase flips, group B at 1 from the start
    "prio_b_hold": [("""    __builtin_amdgcn_s_setprio(0);
  };
  if (!group_b) {""", """    if (!group_b) __builtin_amdgcn_s_setprio(0);
  };
  if (!group_b) {""")],
    "prio_static_b": [("""    __builtin_amdgcn_s_setprio(1);
    // group B's first kAhead pairs""", """    // group B's first kAhead pairs"""),
                      ("""    __builtin_amdgcn_s_setprio(0);
  };
  if (!group_b) {""", """  };
  if (!group_b) {"""),
                      ("""    // group B: phase 2t softmax(t) + K(t+2) staging, phase 2t+1 MFMA
""", """    // group B: phase 2t softmax(t) + K(t+2) staging, phase 2t+1 MFMA
    __builtin_amdgcn_s_setprio(1);
""")],
    # operand ring depth of the MFMA phase (pairs read ahead of their MFMAs; ring = depth + 1); correct results
    "ahead3": [("  constexpr int kAhead = online && !kPersist ? 3 : kAheadDefault;", "  constexpr int kAhead = !kPersist ? 3 : 2;")],
    "ahead2": [("  constexpr int kAhead = online && !kPersist ? 3 : kAheadDefault;", "  constexpr int kAhead = 2;")],
    "ahead4": [("  constexpr int kAhead = online && !kPersist ? 3 : kAheadDefault;", "  constexpr int kAhead = !kPersist ? 4 : 2;")],
    # staging-load probes of the self-attention loop (WRONG results): hotload = every tile's K/V load reads tile t & 1
    # (L2-resident bytes: the HBM part of the load latency gone); noload = no K/V loads after the prologue
    "hotload": [("      kt = t;\n", "      kt = t & 1;\n")],
    "noload": [("""        softmax(t + 1);
        load_tile(t + 2);
      }
      __syncthreads();
    };
    // pairs of tiles""", """        softmax(t + 1);
        if (t < 0) load_tile(t + 2);
      }
      __syncthreads();
    };
    // pairs of tiles"""), ("      if (t + 2 < ntiles) load_tile(t + 3);\n", "      if (t < 0) load_tile(t + 3);\n")],
    # round 5 isolation builds of the self-attention loop (WRONG results; read their probe spans, tools/bench_attn.py
    # --probe, with DEFINES=-DCP25_ATTN_PROBE): noexp = P = bf16(S) without the v_exp (the softmax VALU minus 32 exp per
    # wave and tile); noreads = the MFMA phase's 48 operand reads become empty asm (no LDS read latency or issue)
    "noexp": [("          v[j] = static_cast<__bf16>(__builtin_amdgcn_exp2f(kPre ? sv : fmaf(sv, cs, -m_run[qh])));\n",
               "          v[j] = static_cast<__bf16>(kPre ? sv : fmaf(sv, cs, -m_run[qh]));\n")],
    "noreads": [('      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[n % kR]) : "v"(k_rd_lds), "i"(off));\n',
                 '      asm volatile("; %0 %1 %2" : "=v"(ring[n % kR]) : "v"(k_rd_lds), "i"(off));\n'),
                ('      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(v_rd_lds), "i"(off));\n'
                 '      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(v_rd_lds), "i"(off + 16 * kVStride16));\n',
                 '      asm volatile("; %0 %1 %2" : "=v"(lo) : "v"(v_rd_lds), "i"(off));\n'
                 '      asm volatile("; %0 %1 %2" : "=v"(hi) : "v"(v_rd_lds), "i"(off + 16 * kVStride16));\n')],
    # expdummy: the v_exp runs (its result kept alive) but P = bf16(S) as in noexp: noexp vs expdummy = the exp
    # instruction's own cost, data equal; dmav: V staged by LDS-DMA in the zero-shift form too (correct results)
    "expdummy": [("          v[j] = static_cast<__bf16>(__builtin_amdgcn_exp2f(kPre ? sv : fmaf(sv, cs, -m_run[qh])));\n",
                  "          v[j] = static_cast<__bf16>(kPre ? sv : fmaf(sv, cs, -m_run[qh]));\n"
                  "          { const float e_ = __builtin_amdgcn_exp2f(sv); asm volatile(\"\" ::\"v\"(e_)); }\n")],
    "dmav": [("  constexpr bool kDmaV = kDmaK && online;\n", "  constexpr bool kDmaV = kDmaK;\n")],
    # vsum: the row sums as fp32 VALU adds of the unrounded P (FlashAttention's form) in two per-lane partial chains,
    # reduced over the row's 4 lanes at the end, instead of 4 MFMAs per tile against an all-ones row (different
    # rounding: not bit-identical to the product)
    "vsum": [("""#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb[ks][qh], lsum[qh], 0, 0, 0);
""", ""),
             ("          v[j] = static_cast<__bf16>(__builtin_amdgcn_exp2f(kPre ? sv : fmaf(sv, cs, -m_run[qh])));\n",
              "          const float e_ = __builtin_amdgcn_exp2f(kPre ? sv : fmaf(sv, cs, -m_run[qh]));\n"
              "          lsum[qh][ks] += e_;\n"
              "          v[j] = static_cast<__bf16>(e_);\n"),
             ("    const float l_tot = lsum[qh][0];\n", "    const float l_tot = group4_sum(lsum[qh][0] + lsum[qh][1]);\n"),
             ("      const float inv = 1.f / lsum[qh][0];\n", "      const float inv = 1.f / group4_sum(lsum[qh][0] + lsum[qh][1]);\n")],
    # round 6: cache policy of the self-attention's K / V LDS-DMA (correct results): sc1 / sc0 sc1 / nt loads are
    # L2-served and allocate no L1 line (MI355X_MICROARCH.md); K / V tiles are read once per workgroup
    "kv_sc1": [('      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(tsrc),\n', '      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1 sc1" ::"v"(off), "s"(tsrc),\n')],
    "kv_nt": [('      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(tsrc),\n', '      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1 nt" ::"v"(off), "s"(tsrc),\n')],
    "kv_sc0sc1": [('      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(tsrc),\n', '      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1 sc0 sc1" ::"v"(off), "s"(tsrc),\n')],
    # round 6: the pad lanes of each 288-B LDS row (2 of 18) issue no K / V load at all (exec-masked) instead of
    # re-reading the tile's first 16 B; correct results
    "kv_padskip": [("  int dma_off[5];             // lane source offsets of a full tile, per instruction\n",
                    "  int dma_off[5];             // lane source offsets of a full tile, per instruction\n"
                    "  unsigned dma_ok = 0;\n"),
                   ("    dma_off[j] = cb < 2 * kD ? row * (int)(sl * 2) + cb : 0;\n",
                    "    dma_off[j] = cb < 2 * kD ? row * (int)(sl * 2) + cb : 0;\n"
                    "    dma_ok |= (cb < 2 * kD ? 1u : 0u) << j;\n"),
                   ('      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(tsrc),\n',
                    '      if (dma_ok >> j & 1u)\n'
                    '      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(tsrc),\n')],
    # round 6: the fixed-shift mode (kMode 0) with the shift the row's whole bound, floor(|q_row| kbound), instead of
    # max(b_row - 96, 0): P <= 2 like the online max, and an integer shift, so outputs stay bit-identical to the zero-
    # shift loop (P scaled by an exact power of two). Lab probe of whether P's magnitude moves the power-limited clock
    "dshift": [("      m_run[qh] = fmaxf(sqrtf(group4_sum(qq)) * a.kbound * cs - kTop, 0.f);\n",
                "      m_run[qh] = floorf(sqrtf(group4_sum(qq)) * a.kbound * cs);\n")],
    # round 6: the whole-bound shift pushed further down (rows with b_row <= 30 shift by floor(b_row) + 24 / + 60: P <=
    # 2^-23 / 2^-59): does an even smaller P save more energy? (unit-weight data: b_row ~17). These two and `dshift`
    # patch attn_fwd.hip as it was before the product took the result (kPDrop): build them from that commit's source
    "shift_p24": [("      m_run[qh] = floorf(b_row <= kWhole ? b_row : 126.f - b_row);\n",
                   "      m_run[qh] = floorf(b_row <= 30.f ? b_row + 24.f : (b_row <= kWhole ? b_row : 126.f - b_row));\n")],
    "shift_p60": [("      m_run[qh] = floorf(b_row <= kWhole ? b_row : 126.f - b_row);\n",
                   "      m_run[qh] = floorf(b_row <= 30.f ? b_row + 60.f : (b_row <= kWhole ? b_row : 126.f - b_row));\n")],
    "none": [],
}


def main():
    name, patches = sys.argv[1], sys.argv[2].split(",")
    src = open(os.path.join(CSRC, "attn_fwd.hip")).read()
    for p in patches:
        for old, new in PATCHES[p]:
            assert src.count(old) == 1, (p, old)
            src = src.replace(old, new)
    tmp = f"/tmp/attn_{name}.hip"
    open(tmp, "w").write(src)
    subprocess.check_call(["make", "-s", "-C", CSRC, "-j8"])
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fhip-fp32-correctly-rounded-divide-sqrt",
             "-fno-honor-nans", "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    flags += os.environ.get("DEFINES", "").split()  # e.g. DEFINES=-DCP25_ATTN_PROBE
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", tmp, "-o", f"/tmp/attn_{name}.o"])
    others = [os.path.join(OBJ, f) for f in sorted(os.listdir(OBJ))
              if f.endswith(".o") and f not in ("attn_fwd.o", "attn_w64.o")]
    out = os.path.join(ROOT, "tools", "lab", f"libcp25_{name}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out,
                           f"/tmp/attn_{name}.o", *others])
    print(out)


if __name__ == "__main__":
    main()
