#!/bin/bash
# build a variant library with extra -D flags: build_flags.sh <name> "<flags>"
set -e
cd "$(dirname "$0")"
SRC=../../mh-spgemm_amd/csrc
mkdir -p $1
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $2 -c $SRC/mhs_kernels.hip -o $1/k.o
[ api.o -nt $SRC/mhs_api.cpp ] && [ api.o -nt $SRC/mhs_internal.hpp ] || hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $SRC/mhs_api.cpp -o api.o
[ mmio.o -nt $SRC/mhs_mmio.cpp ] || hipcc -O3 -std=c++17 -fPIC -c $SRC/mhs_mmio.cpp -o mmio.o
hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o $1/libmhspgemm.so $1/k.o api.o mmio.o -lpthread
