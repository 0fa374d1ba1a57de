#!/bin/bash
# Per-kernel VGPR / spills / LDS / occupancy of the gfx950 build (compiler remarks).
# usage: tools/res_usage.sh [file.hip ...]   (default: every .hip)
cd "$(dirname "$0")/../ucla-roms_amd/csrc" || exit 1
files=${@:-*.hip}
for f in $files; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c "$f" -o /tmp/_res.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk '/Function Name:/{n=$5} /VGPRs:/{v=$4} /SGPRs Spill:/{ss=$5} /VGPRs Spill:/{vs=$5} /LDS Size/{l=$6}
         /Occupancy/{o=$5} /LDS Size/{printf "%-58s vgpr=%-4s vspill=%-3s sspill=%-3s lds=%-6s occ=%s\n", substr(n,1,58), v, vs, ss, l, o}'
done
