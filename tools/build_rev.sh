#!/bin/bash
# Build libromsgpu.so of a git revision (A/B against the working tree) into
# ucla-roms_amd/libromsgpu_TAG.so.  usage: tools/build_rev.sh TAG [REV] ["extra flags"]
TAG=$1; REV=${2:-HEAD}; EXTRA=$3
R=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/romsgpu_rev_$TAG
rm -rf $B && mkdir -p $B && (cd $R && git archive $REV ucla-roms_amd/csrc include) | tar -x -C $B
cd $B/ucla-roms_amd/csrc && make -s -j8 FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable $EXTRA" && cp $B/ucla-roms_amd/libromsgpu.so $R/ucla-roms_amd/libromsgpu_$TAG.so && echo "built ucla-roms_amd/libromsgpu_$TAG.so ($REV)"
