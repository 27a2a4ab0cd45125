"""Lab source: the row sums by v_dot2_f32_bf16 on the packed P (16 per tile per lane, in the softmax phase, which has
VALU issue slack beside the partner's MFMA phase) instead of 4 MFMAs against an all-ones row in the MFMA phase (5.9 % of
its MFMA pipe time). Each lane keeps a partial sum of its 16 keys per tile; the 4 lane groups are summed at the end.
Writes /tmp/attn_rsdot2.hip from the product attn_fwd.hip; build with
  python tools/lab/build_tu.py attn_fwd /tmp/attn_rsdot2.hip rsdot2"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc", "attn_fwd.hip")).read()


def rep(old, new, count=1):
    global src
    assert src.count(old) == count, (src.count(old), old[:90])
    src = src.replace(old, new)


rep("""    // keep the whole softmax in this phase: s_barrier orders memory only
    asm volatile("" ::"v"(pb[0][0]), "v"(pb[0][1]), "v"(pb[1][0]), "v"(pb[1][1]));""",
    """    {  // row sums of the bf16 P (this lane's 16 keys of each of its two rows)
      typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
      const bf16x2v one2 = {static_cast<__bf16>(1.f), static_cast<__bf16>(1.f)};
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        float s0 = lsum[qh][0], s1 = 0.f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int w = 0; w < 4; w += 2) {
            s0 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2v{pb[ks][qh][2 * w], pb[ks][qh][2 * w + 1]}, one2, s0, false);
            s1 = __builtin_amdgcn_fdot2_f32_bf16(bf16x2v{pb[ks][qh][2 * w + 2], pb[ks][qh][2 * w + 3]}, one2, s1, false);
          }
        lsum[qh][0] = s0 + s1;
      }
    }
    // keep the whole softmax in this phase: s_barrier orders memory only
    asm volatile("" ::"v"(pb[0][0]), "v"(pb[0][1]), "v"(pb[1][0]), "v"(pb[1][1]));""")
rep("""#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb[ks][qh], lsum[qh], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    static_for<32>""", """    __builtin_amdgcn_sched_barrier(0);
    static_for<32>""")
rep("""      const float inv = 1.f / lsum[qh][0];""", """      const float inv = 1.f / group4_sum(lsum[qh][0]);""")
rep("""    const float l_tot = lsum[qh][0];""", """    const float l_tot = group4_sum(lsum[qh][0]);""")
open("/tmp/attn_rsdot2.hip", "w").write(src)
print("/tmp/attn_rsdot2.hip")
