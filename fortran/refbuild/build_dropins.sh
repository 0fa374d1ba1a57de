#!/bin/bash
# Drop-in build check inside the reference's own source tree (SURVEY.md 8(b),
# callers 1; Work/Makefile:17-24): the case directory's cppdefs.opt and
# param.opt override src/ exactly as the reference's Compile/ copy does, the
# reference's module sources (param, hidden_mpi_vars, dimensions, scalars)
# are preprocessed with cpp | mpc.py (Tools-Roms/mpc_python) and compiled with
# amdflang, and every fortran/dropin/*.F is compiled against those modules
# (plus fortran/roms_gpu_mod.F90).  Output: object files and a symbol table
# under $OUT (default /tmp/roms_dropin_build); nothing is written to the repo
# or to /root/reference.  Container-only: exits 77 when the reference tree
# is absent.
#   usage: fortran/refbuild/build_dropins.sh [CASE_DIR] [OUT]
set -e
REF=${REF:-/root/reference}
[ -d "$REF/src" ] || { echo "reference tree not present"; exit 77; }
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/../.." && pwd)
CASE=${1:-$REF/tests/Filament}
OUT=${2:-/tmp/roms_dropin_build}
FC=${FC:-/opt/rocm/llvm/bin/flang}
MPC=$REF/Tools-Roms/mpc_python/mpc.py
rm -rf "$OUT" && mkdir -p "$OUT" && cd "$OUT"
# case overrides first (the working directory is searched before -I for
# quoted includes when the source comes from stdin), then src/
cp "$CASE/cppdefs.opt" "$CASE/param.opt" .
pp() { cpp -P -traditional -D__IFC -I"$REF/src" < "$1" | python3 "$MPC" > "$2"; }
$FC -c -O2 "$HERE/mpi_f08_shim.f90" -o mpi_f08_shim.o
for m in param hidden_mpi_vars dimensions scalars; do
  pp "$REF/src/$m.F" $m.f
  $FC -c -O2 $m.f -o $m.o
done
$FC -c -O2 "$REPO/fortran/roms_gpu_mod.F90" -o roms_gpu_mod.o
# the glue module first (the routine drop-ins use it), then every routine
pp "$REPO/fortran/dropin/roms_gpu_glue.F" roms_gpu_glue.f
$FC -c -O2 roms_gpu_glue.f -o roms_gpu_glue.o
for f in "$REPO"/fortran/dropin/*.F; do
  b=$(basename "$f" .F)
  [ "$b" = roms_gpu_glue ] && continue
  pp "$f" "dropin_$b.f"
  $FC -c -O2 "dropin_$b.f" -o "dropin_$b.o"
done
# defined subroutine symbols of the drop-ins (what main.F's calls link against)
nm --defined-only dropin_*.o | awk '$2 == "T" {print $3}' | sort > dropin_symbols.txt
echo "built $(ls dropin_*.o | wc -l) drop-ins against $(basename "$CASE") modules in $OUT"
