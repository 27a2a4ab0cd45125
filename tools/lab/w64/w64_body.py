"""Lab: dump the steady-state iteration (136 MFMAs, 64 v_exp) of an attn_fwd_w64 kernel from a .s file."""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
mode = sys.argv[2] if len(sys.argv) > 2 else "1"
name = f"_ZN8cp25attn12_GLOBAL__N_112attn_fwd_w64ILi{mode}ELi0EEEvNS_8AttnArgsE"
i = s.index(name + ":")
f = s[i:s.index(".Lfunc_end", i)]
lines = [l.strip() for l in f.split("\n") if l.strip() and not l.strip().startswith(";") and "implicit-def" not in l
         and not l.strip().startswith(".")]
bars = [k for k, l in enumerate(lines) if "s_barrier" in l]
for a, b in zip(bars, bars[1:]):
    seg = lines[a:b]
    if sum("v_mfma" in l for l in seg) == 136 and sum("v_exp" in l for l in seg) == 64:
        break
c = Counter(l.split()[0] for l in seg)
print(len(seg), sorted(c.items(), key=lambda x: -x[1])[:14])
open("/tmp/body.txt", "w").write("\n".join(seg))
