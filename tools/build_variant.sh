#!/bin/bash
# Build a variant of libmadipm_hip.so with extra compile definitions for ldl.hip (A/B measurements):
#   bash tools/build_variant.sh TAG -DMADIPM_FOLD_GP=32 ...
# -> madipm.jl_amd/madipm_amd/lib/variants/libmadipm_hip_TAG.so (select with MADIPM_LIB=<path>)
set -e
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/madipm.jl_amd/csrc
OBJ=$ROOT/build/obj
OUT=$ROOT/madipm.jl_amd/madipm_amd/lib/variants
mkdir -p $OUT $OBJ/variants
make -s -C $CS >/dev/null
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I$ROOT/include --offload-arch=gfx950 \
  -munsafe-fp-atomics "$@" -c $CS/ldl.hip -o $OBJ/variants/ldl_$TAG.o
OBJS=$(ls $OBJ/*.o | grep -v "/ldl.hip.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libmadipm_hip_$TAG.so $OBJS $OBJ/variants/ldl_$TAG.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo $OUT/libmadipm_hip_$TAG.so
