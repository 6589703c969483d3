#!/bin/bash
# Build ablation variants of libmhspgemm (timing only: results are wrong by design).
#  0 normal, 1 plain LDS store instead of ds_add_f64, 2 no tile lookup,
#  3 no LDS work in the numeric loop, 4 no B loads
set -e
cd "$(dirname "$0")"
SRC=../../mh-spgemm_amd/csrc
for v in "$@"; do
  mkdir -p v$v
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DMHS_NUM_DIAG=$v -c $SRC/mhs_kernels.hip -o v$v/k.o &
done
wait
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $SRC/mhs_api.cpp -o api.o
[ tr.o -nt $SRC/mhs_transpose.hip ] || hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $SRC/mhs_transpose.hip -o tr.o
hipcc -O3 -std=c++17 -fPIC -c $SRC/mhs_mmio.cpp -o mmio.o
for v in "$@"; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o v$v/libmhspgemm.so v$v/k.o tr.o api.o mmio.o -lpthread
done
