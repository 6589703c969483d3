#!/bin/bash
# Build a variant libmhspgemm.so with extra -D flags into tools/var/<name>/ (A/B timing
# via MHS_LIB=tools/var/<name>/libmhspgemm.so).  usage: tools/build_variant.sh <name> -DX=.. ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
out=${OUT:-$ROOT/tools/var}/$name
mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I$ROOT/include "$@" \
    -c $ROOT/mh-spgemm_amd/csrc/mhs_kernels.hip -o $out/mhs_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I$ROOT/include "$@" \
    -x hip -c $ROOT/mh-spgemm_amd/csrc/mhs_api.cpp -o $out/mhs_api.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libmhspgemm.so $out/mhs_kernels.o \
    $ROOT/mh-spgemm_amd/build/mhs_transpose.o $ROOT/mh-spgemm_amd/build/mhs_hbm.o $out/mhs_api.o $ROOT/mh-spgemm_amd/build/mhs_mmio.o -lpthread
rm -f $out/mhs_kernels.o $out/mhs_api.o
echo built $out
