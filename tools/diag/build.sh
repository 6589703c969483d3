#!/bin/bash
# Diagnostic library: per-row, per-phase s_memtime stamps of the numeric rows and the flight
# recorder (-DMHS_ROW_STAMPS=1; read by tools/diag/stamps2.py and tools/diag/flight.py), built
# into tools/diag/stamps/ (git-ignored; travels to the GPU box).  Extra -D flags: "$@".
set -e
cd "$(dirname "$0")"
ROOT=$(cd ../.. && pwd)
SRC=$ROOT/mh-spgemm_amd/csrc
B=$ROOT/mh-spgemm_amd/build
make -s -C $ROOT/mh-spgemm_amd ARCH=gfx950 lib
OUT=${OUT:-stamps}
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -DMHS_ROW_STAMPS=1 "$@" -c $SRC/mhs_kernels.hip -o $OUT/k.o
hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libmhspgemm.so $OUT/k.o $B/mhs_transpose.o $B/mhs_hbm.o $B/mhs_api.o $B/mhs_mmio.o -lpthread
rm -f $OUT/k.o
echo built tools/diag/$OUT/libmhspgemm.so
