#!/bin/bash
# Lab A/B base (round 6): libcp25 with gemm.hip as of git revision $1 (default HEAD), linked with the current product
# objects, for tools/lab/gemm_tail/ab_tail.py. Writes tools/lab/gemm_tail/libcp25_base.so.
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$HERE/../../.."
CSRC="$ROOT/cosmos-predict2.5_amd/csrc"
OBJ="$CSRC/../cosmos_predict2/_lib/obj"
make -s -C "$CSRC"
TMP=$(mktemp -d)
git -C "$ROOT" show "${1:-HEAD}:cosmos-predict2.5_amd/csrc/gemm.hip" > "$TMP/gemm.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fhip-fp32-correctly-rounded-divide-sqrt -Wall \
  -Wno-unused-function -I$ROOT/include -I$CSRC -c "$TMP/gemm.hip" -o "$TMP/gemm.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$HERE/libcp25_base.so" \
  $(ls "$OBJ"/*.o | grep -v -e '/gemm.o$' -e '/attn_w64.o$') "$TMP/gemm.o"
rm -rf "$TMP"
echo "built $HERE/libcp25_base.so"
