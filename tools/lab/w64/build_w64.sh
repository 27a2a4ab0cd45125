#!/bin/bash
# lab: compile attn_w64.hip alone keeping its ISA in /tmp/w64.s, print the ISA summary and the static hazard check
# (the instantiation ILi<mode>ELi0E, mode default 1)
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
CSRC="$HERE/../../../cosmos-predict2.5_amd/csrc"
TMP=$(mktemp -d)
cd "$TMP"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fhip-fp32-correctly-rounded-divide-sqrt -Wall \
  -Wno-unused-function -I$CSRC/../../include -I$CSRC -fno-honor-nans -fno-slp-vectorize -c "$HERE/attn_w64.hip" \
  -o w64.o -save-temps=obj 2>&1 | grep -E "error|warning" | head -20 || true
mv attn_w64-hip-amdgcn-amd-amdhsa-gfx950.s /tmp/w64.s
cd / && rm -rf "$TMP"
python3 "$HERE/w64_isa.py" /tmp/w64.s | grep -A6 "ILi${1:-1}ELi0E"
python3 "$HERE/../../mfma_hazards.py" /tmp/w64.s w64 | grep -v "hazards: 0" || true
