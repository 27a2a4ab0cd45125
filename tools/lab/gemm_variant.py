"""Lab builds of libcp25.so with a text-patched gemm.hip (isolation variants for same-box A/B of the GEMM tile seam;
results are WRONG for every patch except 'none'). The product source is not touched: the patched copy is compiled from
/tmp and linked with the in-tree objects of the other translation units.
usage: python tools/lab/gemm_variant.py <name> <patch>[,<patch>...]  ->  tools/lab/libcp25_<name>.so
patches: nostage (accumulators not written to the LDS C image), nostore (no global C stores), none;
correct-result variants: sc1 (full-tile C stores write-through, dropping the lines from the XCD L2, via a buffer
store with the sc1 policy bit), stagger<N> (workgroup w sleeps ((w >> 3) & 15) x s_sleep N before its first tile, so
the workgroups' tile seams -- and their C-store bursts -- no longer coincide chip-wide), group<G> (kGroupM = G row
tiles per L2 group instead of 8)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc")
OBJ = os.path.join(ROOT, "cosmos-predict2.5_amd", "cosmos_predict2", "_lib", "obj")

PATCHES = {
    "nostage": [("                stj[j][(mq * 128 + 16 * i + r) * 256 + nq * 128] = f2bf(rbf(a));\n",
                 "                if (a == 12345.f) stj[j][(mq * 128 + 16 * i + r) * 256 + nq * 128] = f2bf(rbf(a));\n")],
    "nostore": [("      for (int it = 0; it < 16; ++it) *reinterpret_cast<u32x4*>(crow + (int64_t)it * 16 * ldc) = cv[it];\n",
                 "      for (int it = 0; it < 16; ++it) if (cv[it][0] == 0x12345678u) *reinterpret_cast<u32x4*>(crow + (int64_t)it * 16 * ldc) = cv[it];\n")],
    "sc1": [("    unsigned short* crow = C + (int64_t)(m0 + r0) * ldc + n0 + ch * 8;\n",
             "    unsigned short* crow = C + (int64_t)(m0 + r0) * ldc + n0 + ch * 8;\n"
             "    const auto c_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(C + (int64_t)m0 * ldc + n0), (short)0, 0x7fffffff, 0x00020000);\n"
             "    const int c_off = (r0 * (int)ldc + ch * 8) * 2;\n"),
            ("      for (int it = 0; it < 16; ++it) *reinterpret_cast<u32x4*>(crow + (int64_t)it * 16 * ldc) = cv[it];\n",
             "      for (int it = 0; it < 16; ++it) __builtin_amdgcn_raw_buffer_store_b128(cv[it], c_rsrc, c_off + it * 16 * (int)ldc * 2, 0, 16);\n")],
    "none": [],
}
for _g in (2, 4, 16, 32):  # the L2 grouping of row tiles (tile order only: bit-identical results)
    PATCHES[f"group{_g}"] = [("constexpr int kGroupM = 8;\n", f"constexpr int kGroupM = {_g};\n")]
for _n in (4, 8, 16, 32):
    PATCHES[f"stagger{_n}"] = [("  if (tile >= n_tiles) return;\n",
                                "  if (tile >= n_tiles) return;\n"
                                f"  for (int d = (blockIdx.x >> 3) & 15; d > 0; --d) __builtin_amdgcn_s_sleep({_n});\n")]


def main():
    name, patches = sys.argv[1], sys.argv[2].split(",")
    src = open(os.path.join(CSRC, "gemm.hip")).read()
    for p in patches:
        for old, new in PATCHES[p]:
            assert src.count(old) >= 1, (p, old)
            src = src.replace(old, new)
    tmp = f"/tmp/gemm_{name}.hip"
    open(tmp, "w").write(src)
    subprocess.check_call(["make", "-s", "-C", CSRC, "-j8"])
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fhip-fp32-correctly-rounded-divide-sqrt",
             "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", tmp, "-o", f"/tmp/gemm_{name}.o"])
    others = [os.path.join(OBJ, f + ".o") for f in ("attn_fwd", "dit_ops", "fp8_ops", "unipc", "vae_attn", "vae_ops")]
    out = os.path.join(ROOT, "tools", "lab", f"libcp25_{name}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out,
                           f"/tmp/gemm_{name}.o", *others])
    print(out)


if __name__ == "__main__":
    main()
