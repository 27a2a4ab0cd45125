"""Where a kernel's scratch (spill) instructions sit relative to its loops: tools/asm_spills.py <file.s> <substr>...
Prints, per matching kernel, the basic blocks with scratch loads/stores and the backward branches (loops)."""
import re
import sys

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    for m in re.finditer(r"^(_Z\S*" + re.escape(pat) + r"\S*):\s*;", s, re.M):
        name = m.group(1)
        end = s.index(".Lfunc_end", m.end())
        body = s[m.end():end].split("\n")
        blocks, cur = {}, "entry"
        pos = {}
        for k, l in enumerate(body):
            lb = re.match(r"^(\.LBB\S+):", l)
            if lb:
                cur = lb.group(1)
                pos[cur] = k
                continue
            if "scratch_" in l:
                blocks.setdefault(cur, []).append(l.strip().split()[0])
        loops = []
        for k, l in enumerate(body):
            br = re.search(r"s_c?branch\S*\s+(\.LBB\S+)", l)
            if br and br.group(1) in pos and pos[br.group(1)] < k:
                loops.append((br.group(1), pos[br.group(1)], k))
        print(name, "lines", len(body))
        print("  loops (target, start, end):", loops)
        for b, ops in blocks.items():
            print("  ", b, pos.get(b, 0), len(ops), sorted(set(ops)))
