#!/bin/bash
# Lab build: libcp25 with gemm.hip compiled under -DCP25_LAB_GELU_VALU (the MLP1
# GELU epilogue as gelu_erf in VALU on every element instead of the LDS table), linked with the product objects.
# Writes tools/lab/gelu/libcp25_gelu_valu.so.
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
CSRC="$HERE/../../../cosmos-predict2.5_amd/csrc"
OBJ="$CSRC/../cosmos_predict2/_lib/obj"
make -s -C "$CSRC"
TMP=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fhip-fp32-correctly-rounded-divide-sqrt -Wall \
  -Wno-unused-function -I$CSRC/../../include -I$CSRC -DCP25_LAB_GELU_VALU -c "$CSRC/gemm.hip" -o "$TMP/gemm.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$HERE/libcp25_gelu_valu.so" \
  $(ls "$OBJ"/*.o | grep -v -e '/gemm.o$' -e '/attn_w64.o$') "$TMP/gemm.o"
rm -rf "$TMP"
echo "built $HERE/libcp25_gelu_valu.so"
