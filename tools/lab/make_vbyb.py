"""Lab source: group B stages BOTH the K(t+2) and the V(t+1) tiles by LDS-DMA in its softmax phase (V then has two
phases to land, as K has), group A stages nothing. Assumes k and v share a row stride (the DiT's fused QKV buffer and
the CP path's gathered K|V rows). Writes /tmp/attn_vbyb.hip from the product attn_fwd.hip; build with
  python tools/lab/build_tu.py attn_fwd /tmp/attn_vbyb.hip vbyb"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc", "attn_fwd.hip")).read()


def rep(old, new):
    global src
    assert src.count(old) == 1, old[:90]
    src = src.replace(old, new)


rep("""  constexpr bool kDmaV = kDmaK && online;""", """  constexpr bool kDmaV = false;  // lab: V by group B (kVByB)
  constexpr bool kVByB = kDmaK;""")
rep("""  auto dma_tile = [&](int t, auto BUF) __attribute__((always_inline)) {  // group B: K(t), group A: V(t)
    constexpr int kb = decltype(BUF)::value ? KB1 : 0;
    const char* tsrc = sbase + (int64_t)t * kKBlk * sl * 2;""", """  auto dma_tile = [&](int t, auto BUF, auto ISK) __attribute__((always_inline)) {
    constexpr int kb = decltype(BUF)::value ? KB1 : 0;
    constexpr bool is_k = decltype(ISK)::value;
    const char* tsrc = (is_k ? (const char*)kp : (const char*)vp) + (int64_t)t * kKBlk * sl * 2;""")
rep("""    const unsigned lds0 = (unsigned)(uintptr_t)(lds_char_ptr)(smem + (group_b ? kb : VB0 + (kb ? kVBuf16 : 0)));""",
    """    const unsigned lds0 = (unsigned)(uintptr_t)(lds_char_ptr)(smem + (is_k ? kb : VB0 + (kb ? kVBuf16 : 0)));""")
rep("""  if (kDmaK && group_b) {
    // only tiles that exist: past the last one the row clamp would go negative (the DMA's VGPR offset is unsigned)
    dma_tile(0, B0{});
    if (ntiles > 1) dma_tile(1, B1{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (kDmaV) {
    dma_tile(0, B0{});  // V(0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {""", """  if (kDmaK && group_b) {
    // only tiles that exist: past the last one the row clamp would go negative (the DMA's VGPR offset is unsigned)
    dma_tile(0, B0{}, std::true_type{});
    if (ntiles > 1) dma_tile(1, B1{}, std::true_type{});
    dma_tile(0, B0{}, std::false_type{});  // V(0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (kVByB) {
  } else {""")
rep("""      if (t + 1 < ntiles) {
        if constexpr (kDmaV) {
          dma_tile(t + 1, std::integral_constant<int, par ^ 1>{});  // V(t+1): its buffer is free since the last barrier
          softmax(t + 1);
        } else {""", """      if (t + 1 < ntiles) {
        if constexpr (kVByB) {
          softmax(t + 1);
        } else {""")
rep("""      if constexpr (kDmaK) {
        if (t + 2 < ntiles) dma_tile(t + 2, PAR);  // buffer t & 1: K(t) was consumed in the last two phases
      } else {""", """      if constexpr (kDmaK) {
        if (t + 2 < ntiles) dma_tile(t + 2, PAR, std::true_type{});  // buffer t & 1: K(t) was consumed in the last two phases
        if (t + 1 < ntiles) dma_tile(t + 1, std::integral_constant<int, decltype(PAR)::value ^ 1>{}, std::false_type{});
      } else {""")
open("/tmp/attn_vbyb.hip", "w").write(src)
print("/tmp/attn_vbyb.hip")
