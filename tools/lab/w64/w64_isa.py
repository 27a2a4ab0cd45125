"""Per-kernel ISA summary of a -save-temps .s file: MFMA / v_exp / s_nop / v_mov / accvgpr counts per barrier
segment, register counts and spills (lab tool for attn_fwd_w64)."""
import re
import sys
from collections import Counter


def main(path, pat="w64"):
    s = open(path).read()
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        j = s.index(".Lfunc_end", m.start())
        f = s[m.start():j]
        lines = [l for l in f.split("\n") if l.strip() and not l.strip().startswith(";") and "implicit-def" not in l
                 and not l.strip().startswith(".")]
        meta = s[s.index(".name:           " + name):][:2000] if (".name:           " + name) in s else ""
        regs = {k: re.search(r"\." + k + r":\s+(\d+)", s[s.rfind("- .agpr_count", 0, s.index(".name:           " + name)):s.index(".name:           " + name) + 1500]).group(1)
                for k in ("agpr_count", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size")}
        print(name, regs)
        bars = [0] + [k for k, l in enumerate(lines) if "s_barrier" in l] + [len(lines)]
        for a, b in zip(bars, bars[1:]):
            c = Counter(l.split()[0] for l in lines[a:b])
            print("  seg", a, b, "mfma", c["v_mfma_f32_16x16x32_bf16"], "exp", c["v_exp_f32"], "nop", c["s_nop"],
                  "mov", c["v_mov_b32_e32"] + c["v_mov_b64_e32"], "accrd", c["v_accvgpr_read_b32"],
                  "accwr", c["v_accvgpr_write_b32"], "rl", c["v_readlane_b32"], "wl", c["v_writelane_b32"],
                  "scratch", sum(v for k, v in c.items() if k.startswith("scratch")), "tot", b - a)


if __name__ == "__main__":
    main(*sys.argv[1:])
