#!/bin/bash
# Build an A/B variant of libromsgpu.so with extra compile flags into
# ucla-roms_amd/libromsgpu_TAG.so (load it with ROMS_GPU_LIB=...).
# usage: tools/build_variant.sh TAG "-DROMS_SEG_ROWS=8 -DROMS_SEG_MAXS=16"
TAG=$1; EXTRA=$2
R=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/romsgpu_var_$TAG
rm -rf $B && mkdir -p $B/ucla-roms_amd/csrc $B/include && cp $R/ucla-roms_amd/csrc/*.{hip,h,cpp} $R/ucla-roms_amd/csrc/Makefile $B/ucla-roms_amd/csrc/ && cp $R/include/*.h $B/include/
cd $B/ucla-roms_amd/csrc && make -s -j4 FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable $EXTRA" && cp $B/ucla-roms_amd/libromsgpu.so $R/ucla-roms_amd/libromsgpu_$TAG.so && echo "built ucla-roms_amd/libromsgpu_$TAG.so"
