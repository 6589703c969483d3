#!/bin/bash
# Build flag variants of libmhspgemm: tools/diag/build_flags.sh name "-DFOO=1 -DBAR=2" [name2 "flags2" ...]
set -e
cd "$(dirname "$0")"
SRC=../../mh-spgemm_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $SRC/mhs_api.cpp -o api.o
[ tr.o -nt $SRC/mhs_transpose.hip ] || hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $SRC/mhs_transpose.hip -o tr.o
hipcc -O3 -std=c++17 -fPIC -c $SRC/mhs_mmio.cpp -o mmio.o
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p $name
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c $SRC/mhs_kernels.hip -o $name/k.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o $name/libmhspgemm.so $name/k.o tr.o api.o mmio.o -lpthread
done
