#!/bin/bash
# Lab build of attn_fwd_w64: libcp25 with attn_fwd.hip compiled under -DCP25_LAB_W64 (the w64
# routing and cp25_attn_self_select) plus attn_w64.hip, linked with the product objects of `make -C
# cosmos-predict2.5_amd/csrc`. Writes tools/lab/w64/libcp25_<name>.so for each (name, extra flags) pair:
#   tools/lab/w64/build_lab.sh lab ""  [nd "-DCP25_W64_NODMA"]  [probe "-DCP25_ATTN_PROBE -DCP25_W64_PROBE"] ...
# Load one with `N._LIB_PATH = path` before the first native call (tools/lab/w64/test_attn_w64_gpu.py does).
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
CSRC="$HERE/../../../cosmos-predict2.5_amd/csrc"
OBJ="$CSRC/../cosmos_predict2/_lib/obj"
make -s -C "$CSRC"
B="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fhip-fp32-correctly-rounded-divide-sqrt -Wall \
  -Wno-unused-function -I$CSRC/../../include -I$CSRC"
OBJS=$(ls "$OBJ"/*.o | grep -v -e '/attn_fwd.o$' -e '/attn_w64.o$')
TMP=$(mktemp -d)
pids=()
while [ $# -gt 1 ]; do
  n=$1; f=$2; shift 2
  (
    $B $f -DCP25_LAB_W64 -c "$CSRC/attn_fwd.hip" -o "$TMP/attn_fwd_$n.o"
    $B $f -fno-honor-nans -fno-slp-vectorize -c "$HERE/attn_w64.hip" -o "$TMP/attn_w64_$n.o"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$HERE/libcp25_$n.so" $OBJS "$TMP/attn_fwd_$n.o" \
      "$TMP/attn_w64_$n.o"
    echo "built $HERE/libcp25_$n.so"
  ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
rm -rf "$TMP"
exit $rc
