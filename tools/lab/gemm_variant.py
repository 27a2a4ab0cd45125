"""Lab builds of libcp25.so with a text-patched gemm.hip (isolation variants for same-box A/B of the GEMM tile seam;
results are WRONG for every patch except 'none'). The product source is not touched: the patched copy is compiled from
/tmp and linked with the in-tree objects of the other translation units.
usage: python tools/lab/gemm_variant.py <name> <patch>[,<patch>...]  ->  tools/lab/libcp25_<name>.so
patches: nostage (accumulators not written to the LDS C image), nostore (no global C stores), none"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc")
OBJ = os.path.join(ROOT, "cosmos-predict2.5_amd", "cosmos_predict2", "_lib", "obj")

PATCHES = {
    "nostage": [("              stj[j][(mq * 128 + 16 * i + r) * 256 + nq * 128] = f2bf(y);\n",
                 "              if (y == 12345.f) stj[j][(mq * 128 + 16 * i + r) * 256 + nq * 128] = f2bf(y);\n")],
    "nostore": [("      for (int it = 0; it < 16; ++it) *reinterpret_cast<u32x4*>(crow + (int64_t)it * 16 * ldc) = cv[it];\n",
                 "      for (int it = 0; it < 16; ++it) if (cv[it][0] == 0x12345678u) *reinterpret_cast<u32x4*>(crow + (int64_t)it * 16 * ldc) = cv[it];\n")],
    "none": [],
}


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
