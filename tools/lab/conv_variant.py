"""Lab builds of libcp25.so with a text-patched vae_ops.hip (isolation variants of the halo conv's LDS-DMA sources,
for same-box A/B with tools/bench_conv.py; results are WRONG for every patch except 'none'). The product source is not
touched: the patched copy is compiled from /tmp and linked with the in-tree objects of the other translation units.
usage: python tools/lab/conv_variant.py <name> <patch>[,<patch>...]  ->  tools/lab/libcp25_<name>.so
patches: wcontig (each weight DMA instruction reads 1 KiB contiguous: the bytes of a stage-major weight layout),
         hcontig (each halo DMA instruction reads 32 pixels x 32 B contiguous: a channel-blocked activation layout),
         (the tw32 / tw64 tile-width patches of profiles/r3/conv/tile_width_ab.log were applied to the source before 16 x 32
         tiles became the default; see git history)
         none"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc")
OBJ = os.path.join(ROOT, "cosmos-predict2.5_amd", "cosmos_predict2", "_lib", "obj")

PATCHES = {
    "wcontig": [("      if (co < a.Cout) off = (co * a.KT * 9 + tap) * a.Cin + 8 * half;\n",
                 "      if (co < a.Cout) off = wi_ * 512 + lane * 8;\n")],
    "hcontig": [("          off = (hi * a.Win + wi) * a.Cin + 8 * half;\n",
                 "          off = (hi * a.Win + wi) * 16 + 8 * half;\n")],
    "none": [],
}


def main():
    name, patches = sys.argv[1], sys.argv[2].split(",")
    src = open(os.path.join(CSRC, "vae_ops.hip")).read()
    for p in patches:
        for old, new in PATCHES[p]:
            assert src.count(old) == 1, (p, old)
            src = src.replace(old, new)
    tmp = f"/tmp/vae_ops_{name}.hip"
    open(tmp, "w").write(src)
    subprocess.check_call(["make", "-s", "-C", CSRC, "-j8"])
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fhip-fp32-correctly-rounded-divide-sqrt",
             "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", tmp, "-o", f"/tmp/vae_ops_{name}.o"])
    others = [os.path.join(OBJ, f + ".o") for f in ("attn_fwd", "dit_ops", "fp8_ops", "gemm", "unipc", "vae_attn")]
    out = os.path.join(ROOT, "tools", "lab", f"libcp25_{name}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out,
                           f"/tmp/vae_ops_{name}.o", *others])
    print(out)


if __name__ == "__main__":
    main()
