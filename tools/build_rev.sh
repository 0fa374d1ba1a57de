#!/bin/bash
# Build libromsgpu.so from a git revision's sources into
# ucla-roms_amd/libromsgpu_<tag>.so (an A/B arm: ROMS_GPU_LIB=..., tools/gpu.sh ab lib:<tag>).
# usage: bash tools/build_rev.sh REV TAG
set -e
REV=$1; TAG=$2
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/romsrev_$TAG
rm -rf $W && mkdir -p $W
git -C $R archive $REV ucla-roms_amd/csrc include | tar -x -C $W
make -s -j8 -C $W/ucla-roms_amd/csrc OUT=$R/ucla-roms_amd/libromsgpu_$TAG.so
echo built $R/ucla-roms_amd/libromsgpu_$TAG.so from $(git -C $R rev-parse --short $REV)
