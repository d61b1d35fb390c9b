#!/bin/bash
# Replays the round-5 wrong-pivot failure of the assembly's LDS source path (gpurun_out/r6_q, r6_r:
# test_batched_leaf_columns_parity[100-800-0-128], "1 pivots off; worst k=899 gpu=-1287.97...").
# Cause: the tile's source count rides in gchk's top 16 bits and was read back with a SIGNED shift;
# dense_k2(100, 800)'s root has a tile of 49,344 >= 2^15 sources, which read negative and summed
# nothing.  This builds ldl.hip with the old signed read as a variant and runs the windowed-path test
# with every tile of <= 12 windows on the path (MADIPM_ASM_LDS_WIN=12): the variant must fail with the
# k=899 signature, the committed build must pass.
#   bash tools/repro_r5_signed_count.sh build      (here: hipcc cross-compiles the variant .so, which travels)
#   bash tools/repro_r5_signed_count.sh run TAG    (GPU box)
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
V=$ROOT/madipm.jl_amd/madipm_amd/lib/variants/libmadipm_hip_signed_count.so
if [ "$1" = "build" ]; then
SRC=$ROOT/build/repro_signed/ldl.hip; mkdir -p $(dirname $SRC)
sed 's/int ns = (int)((uint64_t)tl.gchk >> 48);/int ns = (int)(tl.gchk >> 48);/' $ROOT/madipm.jl_amd/csrc/ldl.hip > $SRC
grep -q 'int ns = (int)(tl.gchk >> 48);' $SRC || { echo "patch did not apply"; exit 1; }
cp $ROOT/madipm.jl_amd/csrc/*.hpp $(dirname $SRC)/
mkdir -p $(dirname $V)
make -s -C $ROOT/madipm.jl_amd/csrc >/dev/null || exit 1
OBJS=$(ls $ROOT/build/obj/*.o | grep -v "/ldl.hip.o$")
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -I$ROOT/include --offload-arch=gfx950 -munsafe-fp-atomics -c $SRC -o $(dirname $SRC)/ldl.o \
  && /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $V $OBJS $(dirname $SRC)/ldl.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
  || { echo "variant build failed"; exit 1; }
echo $V; exit 0
fi
TAG=${2:-repro_signed}; OUT=gpurun_out/$TAG; mkdir -p $OUT
[ -f $V ] || { echo "build the variant first: bash tools/repro_r5_signed_count.sh build"; exit 1; }
T="tests/test_asm_lds_gpu.py::test_asm_lds_windows_bitwise[dense_100_800]"
MADIPM_LIB=$V timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu "$T" > $OUT/signed_variant.log 2>&1
rc=$?
grep -E "pivots differ|passed|failed" $OUT/signed_variant.log | head -5
[ $rc -eq 1 ] || { echo "expected the signed-count variant to fail (rc=$rc)"; exit 1; }
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu "$T" > $OUT/committed.log 2>&1 \
  || { echo "committed build failed"; tail -20 $OUT/committed.log; exit 1; }
tail -1 $OUT/committed.log
