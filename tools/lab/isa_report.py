#!/usr/bin/env python3
"""Per-kernel ISA report of a HIP source built for gfx950: VGPRs, spills, and the scratch / vmcnt(0) instructions
inside loop blocks (what a 256-VGPR tile loop must not contain). Usage: isa_report.py file.hip [name-filter] [hipcc args]"""
import re, subprocess, sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
extra = sys.argv[3:]
cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fhip-fp32-correctly-rounded-divide-sqrt',
       '-Iinclude', '-fno-honor-nans', '-fno-slp-vectorize', '--cuda-device-only', '-S', src, '-o', '/tmp/isa_report.s',
       '-Rpass-analysis=kernel-resource-usage'] + extra
r = subprocess.run(cmd, capture_output=True, text=True)
res, cur = {}, None
for line in r.stderr.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = m.group(1); res[cur] = {}
        continue
    m = re.search(r'(VGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\d+)', line)
    if m and cur:
        res[cur][m.group(1).split(' [')[0]] = int(m.group(2))
if r.returncode:
    print(r.stderr[-3000:]); sys.exit(1)
s = open('/tmp/isa_report.s').read()
for name, info in res.items():
    if flt not in name:
        continue
    i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
    body = s[i:j].split('\n')
    inloop = False; nscr = nvm0 = 0
    for l in body:
        if re.match(r'^\.LBB', l):
            inloop = 'Loop' in l
        if inloop and 'scratch_' in l: nscr += 1
        if inloop and re.search(r's_waitcnt vmcnt\(0\)', l): nvm0 += 1
    print(f"{name[:70]:70s} vgpr {info.get('VGPRs')} spill {info.get('VGPRs Spill')} sspill {info.get('SGPRs Spill')} "
          f"lds {info.get('LDS Size')} | in-loop scratch {nscr} vmcnt(0) {nvm0}")
