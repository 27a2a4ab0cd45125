"""Static check of asm-MFMA operand hazards the compiler does not pad (round 6, attn_fwd_w64): a VALU instruction
(v_mov, v_accvgpr_write, v_cvt, ...) writing a register that an MFMA within the next `need` wait states reads as
A / B / C. Wait states: s_nop N counts N + 1, any other instruction 1. Usage: mfma_hazards.py file.s [kernel-substring]
Prints the hazards; exit status 1 if any."""
import re
import sys


def regs(tok):
    """'v[4:7]' -> {v4..v7}, 'a12' -> {a12}, 'v3' -> {v3}; others -> empty"""
    m = re.match(r"([va])\[(\d+):(\d+)(?:\+(\d+))?\]", tok)
    if m:
        lo = int(m.group(2))
        hi = int(m.group(3)) + (int(m.group(4)) if m.group(4) else 0)
        if m.group(4):  # a[0x80:0x80+3] style is printed as decimal here
            hi = lo + int(m.group(4))
        return {f"{m.group(1)}{i}" for i in range(lo, hi + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    if m:
        return {tok}
    return set()


def parse_ops(line):
    ins = line.split(None, 1)
    if len(ins) < 2:
        return ins[0], []
    ops = [o.strip() for o in ins[1].split(",")]
    return ins[0], ops


def check(lines, need=2):
    found = []
    hist = []  # (index, written regs, text) of recent VALU writes, with wait states since
    for k, raw in enumerate(lines):
        line = raw.strip()
        if not line or line.startswith((";", ".")) or line.endswith(":"):
            continue
        op, ops = parse_ops(line)
        if op.startswith("v_mfma"):
            read = set()
            for o in ops[1:]:
                read |= regs(o.replace("0x", "").replace(" ", "")) if "0x" not in o else regs(
                    re.sub(r"0x([0-9a-f]+)", lambda m: str(int(m.group(1), 16)), o))
            for ws, wr, txt in hist:
                if ws < need and wr & read:
                    found.append((k, line, txt, ws))
        ws_add = 1
        if op == "s_nop":
            ws_add = int(ops[0], 0) + 1
        hist = [(ws + ws_add, wr, txt) for ws, wr, txt in hist if ws + ws_add < need]
        if op.startswith("v_") and not op.startswith("v_mfma") and ops:
            hist.append((0, regs(ops[0]), line))
    return found


def main(path, pat=""):
    s = open(path).read()
    bad = 0
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M):
        if pat not in m.group(1):
            continue
        body = s[m.start():s.index(".Lfunc_end", m.start())].split("\n")
        f = check(body)
        print(m.group(1), "hazards:", len(f))
        for k, a, b, ws in f[:10]:
            print("   ", b, "->", a, "(wait states", ws, ")")
        bad += len(f)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main(*sys.argv[1:])
