"""Lab build of libcp25.so with one translation unit compiled from another source (e.g. a saved earlier version of
the product file, for same-box A/B runs); the other units are the in-tree objects.
usage: python tools/lab/build_tu.py <unit: attn_fwd|vae_ops|gemm|...> <source.hip> <name>  ->  tools/lab/libcp25_<name>.so"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc")
OBJ = os.path.join(ROOT, "cosmos-predict2.5_amd", "cosmos_predict2", "_lib", "obj")
UNITS = ("attn_fwd", "dit_ops", "fp8_ops", "gemm", "unipc", "vae_attn", "vae_ops")


def main():
    unit, src, name = sys.argv[1:4]
    assert unit in UNITS, unit
    subprocess.check_call(["make", "-s", "-C", CSRC, "-j8"])
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-fhip-fp32-correctly-rounded-divide-sqrt",
             "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    if unit in ("attn_fwd", "vae_attn"):  # the Makefile's per-unit flags
        flags += ["-fno-honor-nans", "-fno-slp-vectorize"]
    obj = f"/tmp/{unit}_{name}.o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", src, "-o", obj])
    others = [os.path.join(OBJ, u + ".o") for u in UNITS if u != unit]
    out = os.path.join(ROOT, "tools", "lab", f"libcp25_{name}.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, obj, *others])
    print(out)


if __name__ == "__main__":
    main()
