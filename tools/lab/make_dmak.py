"""Lab source: the self-attention's K tiles (group B) staged straight into their padded LDS rows by LDS-DMA instead of
through registers (the staging-load probe put the register path at 4.7 % of the launch). Writes /tmp/attn_dmak.hip from
the product attn_fwd.hip; build with tools/lab/build_tu.py attn_fwd /tmp/attn_dmak.hip dmak.
Instruction j of group-B wave w covers K-buffer bytes [1024 (w + 4 j), +1024) (18 per 64 x 288-B tile: waves 0-1 issue
5, waves 2-3 issue 4); lane l moves the 16 B at byte 16 l of it: row b / 288, column b % 288 (columns >= 256 are the
row padding: they re-read the tile's first 16 B). Rows past Lk on the ragged tile read row rows - 1 (their scores are
masked to -inf). Only the per-block kernels (not the persistent form) take this path.
usage: make_dmak.py [kv|mode]   (mode: K always, V in the online-max form only)   (kv: group A's V tiles too, issued at the start of its softmax phase, waited before the
barrier that closes it; rows past Lk read row rows - 1, finite, under P = 0) -> /tmp/attn_dmak[v].hip"""
import os
import sys

KV = len(sys.argv) > 1 and sys.argv[1] in ("kv", "mode")
MODE = len(sys.argv) > 1 and sys.argv[1] == "mode"

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc", "attn_fwd.hip")).read()


def rep(old, new):
    global src
    assert src.count(old) == 1, old[:90]
    src = src.replace(old, new)


rep("""  char* const k_wr = smem + srow * kKStride16 + sch * 16;
""", """  char* const k_wr = smem + srow * kKStride16 + sch * 16;
  constexpr bool kDmaK = !kPersist;
  const int wb = (wave_u & 3);  // wave within its group
  int koff[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int bb = 1024 * (wb + 4 * j) + 16 * lane;
    const int row = bb / kKStride16, cb = bb - row * kKStride16;
    koff[j] = cb < 2 * kD ? row * (int)(sl * 2) + cb : 0;
  }
  auto dma_k = [&](int t, auto BUF) __attribute__((always_inline)) {
    constexpr int kb = decltype(BUF)::value ? KB1 : 0;
    const char* tile = (const char*)(group_b ? kp : vp) + (int64_t)t * kKBlk * sl * 2;
    const int rows = min(Lk - t * kKBlk, kKBlk);
    const unsigned lds0 = (unsigned)(uintptr_t)(lds_char_ptr)(smem + (group_b ? kb : VB0 + (kb ? kVBuf16 : 0)));
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (wb + 4 * j >= 18) break;  // wave-uniform
      int off = koff[j];
      if (__builtin_expect(rows < kKBlk, 0)) {
        const int bb = 1024 * (wb + 4 * j) + 16 * lane;
        const int row = bb / kKStride16, cb = bb - row * kKStride16;
        off = cb < 2 * kD ? min(row, rows - 1) * (int)(sl * 2) + cb : 0;
      }
      asm volatile("s_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(tile),
                   "s"(lds0 + 1024 * (wb + 4 * j)) : "memory");
    }
  };
""")
# prologue (the m16 kernel's; its text is unique with the "written in phase 0" comment)
rep("""  load_tile(0);
  if (group_b) write_k(B0{}); else write_v(B0{});
  if (group_b) {
    load_tile(1);
    write_k(B1{});
    load_tile(2);  // written in phase 0
  } else {
    load_tile(1);  // written in phase 1
  }
  __syncthreads();""", """  if (kDmaK && group_b) {
    dma_k(0, B0{});
    dma_k(1, B1{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    load_tile(0);
    if (group_b) write_k(B0{}); else write_v(B0{});
    if (group_b) {
      load_tile(1);
      write_k(B1{});
      load_tile(2);  // written in phase 0
    } else {
      load_tile(1);  // written in phase 1
    }
  }
  __syncthreads();""")
rep("""    auto step = [&](auto PAR, int t) __attribute__((always_inline)) {
      if (t + 2 < ntiles) write_k(PAR);
      softmax(t);
      if (t + 2 < ntiles) load_tile(t + 3);""", """    auto step = [&](auto PAR, int t) __attribute__((always_inline)) {
      if constexpr (kDmaK) {
        if (t + 2 < ntiles) dma_k(t + 2, PAR);  // buffer t & 1: K(t) was consumed in the last two phases
      } else {
        if (t + 2 < ntiles) write_k(PAR);
      }
      softmax(t);
      if constexpr (!kDmaK) {
        if (t + 2 < ntiles) load_tile(t + 3);
      }""")
rep("""      mfma_phase(PAR, std::true_type{});
      __syncthreads();
    };""", """      mfma_phase(PAR, std::true_type{});
      if constexpr (kDmaK) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K(t+2) landed before A reads it
      __syncthreads();
    };""")
if KV:
    rep("""  if (kDmaK && group_b) {
    dma_k(0, B0{});
    dma_k(1, B1{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {""", """  if (kDmaK && group_b) {
    dma_k(0, B0{});
    dma_k(1, B1{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (kDmaK) {
    dma_k(0, B0{});  // V(0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {""")
    rep("""      if (t + 1 < ntiles) {
        write_v(std::integral_constant<int, par ^ 1>{});  // drains under the softmax VALU
        softmax(t + 1);
        load_tile(t + 2);
      }
      __syncthreads();""", """      if (t + 1 < ntiles) {
        if constexpr (kDmaK) {
          dma_k(t + 1, std::integral_constant<int, par ^ 1>{});  // V(t+1): buffer free since the last barrier
          softmax(t + 1);
        } else {
          write_v(std::integral_constant<int, par ^ 1>{});  // drains under the softmax VALU
          softmax(t + 1);
          load_tile(t + 2);
        }
      }
      if constexpr (kDmaK) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();""")
if MODE:
    rep("""  } else if (kDmaK) {
    dma_k(0, B0{});  // V(0)""", """  } else if (kDmaV) {
    dma_k(0, B0{});  // V(0)""")
    rep("""        if constexpr (kDmaK) {
          dma_k(t + 1, std::integral_constant<int, par ^ 1>{});  // V(t+1): buffer free since the last barrier""",
        """        if constexpr (kDmaV) {
          dma_k(t + 1, std::integral_constant<int, par ^ 1>{});  // V(t+1): buffer free since the last barrier""")
    rep("""      if constexpr (kDmaK) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();""", """      if constexpr (kDmaV) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();""")
    rep("""  constexpr bool kDmaK = !kPersist;
""", """  constexpr bool kDmaK = !kPersist;
  constexpr bool kDmaV = kDmaK && kMode == 2;  // V too in the online form (zero shift: K only, measured)
""")
out = "/tmp/attn_dmakmode.hip" if MODE else ("/tmp/attn_dmakv.hip" if KV else "/tmp/attn_dmak.hip")
open(out, "w").write(src)
print(out)
