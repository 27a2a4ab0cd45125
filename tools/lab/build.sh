#!/bin/bash
# Lab builds of libcp25.so with extra attn_fwd.hip defines, for same-box A/B runs of
# tools/bench_attn.py --lib tools/lab/libcp25_<name>.so (not part of the product build).
# usage: [SRC=/tmp/x.hip] tools/lab/build.sh <name> [-DFOO ...]  (SRC: the attention source; default the product
# attn_fwd.hip; a generated variant or an earlier build from git history, tools/lab/README.md)
set -e
cd "$(dirname "$0")/../.."
make -C cosmos-predict2.5_amd/csrc -j8 >/dev/null
name=$1; shift
OBJ=cosmos-predict2.5_amd/cosmos_predict2/_lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-honor-nans -fno-slp-vectorize -Iinclude -Icosmos-predict2.5_amd/csrc "$@" -c ${SRC:-cosmos-predict2.5_amd/csrc/attn_fwd.hip} -o /tmp/attn_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab/libcp25_$name.so /tmp/attn_$name.o \
  $OBJ/dit_ops.o $OBJ/fp8_ops.o $OBJ/gemm.o $OBJ/unipc.o $OBJ/vae_attn.o $OBJ/vae_ops.o
echo tools/lab/libcp25_$name.so
