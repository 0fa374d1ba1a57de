#!/bin/bash
# Per-kernel VGPR / scratch / occupancy of the gfx950 build (compiler remarks).
cd "$(dirname "$0")/../ucla-roms_amd/csrc" || exit 1
for f in *.hip; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c "$f" -o /tmp/_res.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk '/Function Name:/{n=$5} /VGPRs:/{v=$4} /ScratchSize/{s=$5} /Occupancy/{printf "%-60s vgpr=%-4s scratch=%-4s occ=%s\n", n, v, s, $5}'
done
