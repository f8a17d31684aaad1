#!/bin/bash
# Measurement build of the library with one translation unit recompiled under extra defines:
#   UNIT=corr_bwd_strip DEFS="-DPWC_BWD_GEO4=32,3,28,8" bash tools/build_variant.sh abl/b4cs8
# -> abl/b4cs8/libpwc_hotpath.so (select with PWC_HOTPATH_LIB=...).  Needs the in-tree objects
# (make -C pwc-net_pytorch_amd/csrc) first.
set -e
OUTDIR=$1
UNIT=${UNIT:?unit}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/pwc-net_pytorch_amd/build/obj
mkdir -p $OUTDIR
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -ffp-contract=fast-honor-pragmas \
  -munsafe-fp-atomics -fvisibility=hidden -fno-slp-vectorize $DEFS -c -o $OUTDIR/$UNIT.o \
  $ROOT/pwc-net_pytorch_amd/csrc/$UNIT.hip
objs=$(ls $OBJ/*.o | grep -v "/$UNIT.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUTDIR/libpwc_hotpath.so $objs $OUTDIR/$UNIT.o
rm -f $OUTDIR/$UNIT.o
