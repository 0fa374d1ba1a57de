#!/bin/bash
# Build an A/B variant of libromsgpu.so with extra compile flags into
# ucla-roms_amd/libromsgpu_<tag>.so (loaded with ROMS_GPU_LIB=...).
# usage: bash tools/build_variant.sh TAG "-DFOO=1 -DBAR=2"
set -e
TAG=$1; EXTRA=$2
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/romsvar_$TAG
rm -rf $W && mkdir -p $W/lib/csrc $W/include
cp $R/ucla-roms_amd/csrc/*.h $R/ucla-roms_amd/csrc/*.hip $R/ucla-roms_amd/csrc/*.cpp $R/ucla-roms_amd/csrc/Makefile $W/lib/csrc/
cp $R/include/roms_gpu.h $W/include/
cd $W/lib/csrc
make -s -j8 FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable $EXTRA" \
     OUT=$R/ucla-roms_amd/libromsgpu_$TAG.so
echo built $R/ucla-roms_amd/libromsgpu_$TAG.so
