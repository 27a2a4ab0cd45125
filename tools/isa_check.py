#!/usr/bin/env python3
"""Static checks of the gfx950 ISA of a HIP source (hipcc --cuda-device-only -S): per kernel, VGPRs / spills (the
compiler's resource remarks), in-loop scratch and vmcnt(0), s_nop count, and LDS-read races: an instruction that reads
or writes a VGPR while an LDS read into it is still in flight (not yet retired by an s_waitcnt lgkmcnt, counted in
issue order, joined over the control-flow graph's paths). The hand-scheduled kernels issue ds_reads from inline asm whose destinations the compiler does not know
are written asynchronously; if such an asm output is dead (e.g. its MFMA was eliminated) the register allocator may
hand the register to another value while the read is in flight -- a silent wrong result this check catches.
usage: python tools/isa_check.py file.hip [name-filter]   (exit 1 on any race)"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


_ASM_CACHE = {}


def compile_asm(src, out=None, extra=()):
    """(asm text, resource remarks per kernel) of src; cached per (source path, mtime, extra flags) in this process,
    so several checks of one source compile it once."""
    key = (os.path.abspath(src), os.path.getmtime(src), tuple(extra))
    if key not in _ASM_CACHE:
        _ASM_CACHE[key] = _compile_asm(src, out or f"/tmp/isa_check_{os.getpid()}_{os.path.basename(src)}.s", extra)
    return _ASM_CACHE[key]


def _compile_asm(src, out, extra=()):
    unit_flags = ["-fno-honor-nans", "-fno-slp-vectorize"] if os.path.basename(src).startswith(("attn_fwd", "vae_attn")) \
        else []  # the Makefile's per-unit flags
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "cosmos-predict2.5_amd", "csrc"), *unit_flags,
           "--cuda-device-only", "-S", src, "-o", out, "-Rpass-analysis=kernel-resource-usage", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-3000:])
    res, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
            continue
        m = re.search(r"(VGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            res[cur][m.group(1).split(" [")[0]] = int(m.group(2))
    return open(out).read(), res


_REG = re.compile(r"(?<![\w.])([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def _regs(text):
    """VGPRs and AGPRs named in an operand text, as ('v', n) / ('a', n); source modifiers (-v1, |v1|, neg(..), abs(..))
    and op_sel suffixes do not hide a register."""
    out = set()
    for kind, lo, hi, one in _REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def _merge(a, b):
    """Join of two in-flight LDS-read queues (oldest first), aligned at the newest entry: an lgkmcnt(n) wait keeps the
    newest n entries, so entry k from the end means the same thing on both paths."""
    n = max(len(a), len(b))
    a = [set()] * (n - len(a)) + list(a)
    b = [set()] * (n - len(b)) + list(b)
    return [x | y for x, y in zip(a, b)][-32:]


def analyse(asm, name):
    """Per kernel: races found by a dataflow over the control-flow graph (each instruction's in-flight LDS reads are the
    join over its predecessors: fall-through, unless the previous instruction is an unconditional branch or the end of
    the program, and every branch to its label), s_nop counts (whole kernel and inside loops), and in-loop scratch /
    vmcnt(0) counts."""
    i = asm.index(name + ":")
    j = asm.index(".Lfunc_end", i)
    lines = asm[i:j].split("\n")
    ins, labels, nops, m0nops = [], {}, 0, 0
    inloop, scr, vm0, lnops = False, 0, 0, 0
    for l in lines:
        s = l.strip()
        if not s or s.startswith(";"):
            continue
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            inloop = "Loop" in l
            labels[m.group(1)] = len(ins)
            continue
        if s.startswith("."):
            continue
        t = s.replace(",", " ").split()
        op = t[0]
        if inloop and op.startswith("scratch_"):
            scr += 1
        if inloop and op == "s_waitcnt" and "vmcnt(0)" in s:
            vm0 += 1
        if op == "s_nop":
            if ins and ins[-1][0] == "s_mov_b32" and ins[-1][1][1] == "m0":
                m0nops += 1  # the M0-write -> LDS-DMA separation the DMA asm carries, not a hazard pad
            else:
                nops += 1
                lnops += inloop
        ins.append((op, t, s))
    succ = []
    for k, (op, t, s) in enumerate(ins):
        nxt = []
        if op.startswith("s_cbranch") or op == "s_branch":
            if len(t) > 1 and t[1] in labels:
                nxt.append(labels[t[1]])
        if op not in ("s_branch", "s_endpgm", "s_setpc_b64") and k + 1 < len(ins):
            nxt.append(k + 1)
        succ.append(nxt)
    state = [None] * len(ins)
    state[0] = []
    work = [0]
    races = set()
    while work:
        k = work.pop()
        op, t, s = ins[k]
        pending = [set(x) for x in state[k]]
        live = set().union(*pending) if pending else set()
        ops = s.split(None, 1)[1] if " " in s else ""
        if live and _regs(ops) & live:  # any operand, a ds_read's address and destination included
            races.add((k, s))
        if op.startswith("ds_read"):
            pending.append(_regs(t[1]))
        elif op.startswith(("ds_", "s_load", "s_buffer_load")):
            pending.append(set())
        elif op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", s)
            if m:
                n = int(m.group(1))
                pending = pending[len(pending) - n:] if len(pending) > n else pending
        for q in succ[k]:
            new = pending if state[q] is None else _merge(state[q], pending)
            if state[q] is None or new != state[q]:
                state[q] = new
                work.append(q)
    # M0 outside the inline asm: the attention's DMA asm writes M0 without declaring it (a reserved register the
    # compiler never allocates; a clobber of it is ignored), so any compiler-emitted instruction naming M0 in such a
    # kernel (compiler-visible LDS-DMA, s_sendmsg, movrel indexing) could see or leave a value the asm relies on
    m0_uses, in_asm = [], False
    for l in lines:
        s = l.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
        elif s.startswith(";;#ASMEND"):
            in_asm = False
        elif not in_asm and s and not s.startswith((";", ".")) and re.search(r"(?<![\w])m0(?![\w])", s):
            m0_uses.append(s)
    return {"races": [s for _, s in sorted(races)], "nops": nops, "inloop_nops": lnops, "m0_nops": m0nops,
            "inloop_scratch": scr, "inloop_vmcnt0": vm0, "m0_uses": m0_uses}


def check(src, flt=""):
    asm, res = compile_asm(src)
    out = {}
    for name in re.findall(r"^(_Z\S+):", asm, re.M):
        if flt in name:
            out[name] = dict(res.get(name, {}), **analyse(asm, name))
    return out


if __name__ == "__main__":
    rep = check(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    bad = 0
    for name, r in rep.items():
        bad += len(r["races"])
        print(f"{name[:72]:72s} vgpr {r.get('VGPRs')} spill {r.get('VGPRs Spill')} | in-loop scratch "
              f"{r['inloop_scratch']} vmcnt(0) {r['inloop_vmcnt0']} | s_nop {r['nops']} (+{r['m0_nops']} M0) | LDS races {len(r['races'])}"
              f" | compiler M0 uses {len(r['m0_uses'])}")
        for s in r["races"][:3]:
            print("    race:", s[:100])
    sys.exit(1 if bad else 0)
