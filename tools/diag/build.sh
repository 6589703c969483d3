#!/bin/bash
# Diagnostic library: per-row, per-phase s_memtime stamps of the numeric rows
# (-DMHS_ROW_STAMPS=1; read by tools/diag/stamps*.py).  Built into tools/diag/v9.
set -e
cd "$(dirname "$0")"
SRC=../../mh-spgemm_amd/csrc
mkdir -p v9
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DMHS_ROW_STAMPS=1 -c $SRC/mhs_kernels.hip -o v9/k.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $SRC/mhs_api.cpp -o api.o
[ tr.o -nt $SRC/mhs_transpose.hip ] || hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $SRC/mhs_transpose.hip -o tr.o
hipcc -O3 -std=c++17 -fPIC -c $SRC/mhs_mmio.cpp -o mmio.o
hipcc --offload-arch=gfx950 -shared -fPIC -o v9/libmhspgemm.so v9/k.o tr.o api.o mmio.o -lpthread
