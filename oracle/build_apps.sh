#!/usr/bin/env bash
# Build the reference's float MPI applications twice, unchanged, from their sources in place under
# /root/reference (nothing is copied into the repository; outputs go to oracle/_ref/apps/ only):
#   <app>_ref   : app + the reference codec impl/dataCompression.c (the CPU baseline, as impl/Makefile)
#   <app>_dcamd : app + libdcamd (this repo's include/dataCompression.h, -ldcamd) -- the drop-in check
# The bound is the reference's compile-time macro; the generated header of build_ref.sh redefines it
# for the _ref build, and -DabsErrorBound / DC_ABS_ERROR_BOUND select it for the _dcamd build.
# `-iquote <dir> -I-` keeps the compiler from taking the header that sits next to the app source.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
REPO=$(cd "$HERE/.." && pwd)
OUT="$HERE/_ref/apps"
MPI=${MPI:-/opt/conda}
BOUND=${BOUND:-0.001}
if [ ! -f "$REF/impl/pingpong.c" ] || [ ! -x "$MPI/bin/mpicc" ]; then
  echo "build_apps: reference or mpicc not present, skipping"; exit 0
fi
tag=$(python3 -c "print('%g' % $BOUND)")
gen="$HERE/_ref/gen_$tag"
mkdir -p "$OUT" "$gen"
printf '#include "%s/impl/dataCompression.h"\n#undef absErrorBound\n#define absErrorBound %s\n' "$REF" "$BOUND" > "$gen/dataCompression.h"
LIB="$REPO/data-compression_amd/lib"
STDCXX=$(g++ -print-file-name=libstdc++.so)     # the conda MPI wrapper's -L would pick an older one
for app in pingpong himenoBMTxps; do
  MPICH_CC=gcc "$MPI/bin/mpicc" -O3 -ffp-contract=off -w -iquote "$gen" -I- -I"$gen" -I"$REF/impl" \
      "$REF/impl/$app.c" "$REF/impl/dataCompression.c" -o "$OUT/${app}_ref" -lz -lm
  MPICH_CC=gcc "$MPI/bin/mpicc" -O3 -w -DabsErrorBound="$BOUND" -iquote "$REPO/include" -I- -I"$REPO/include" \
      -I"$REF/impl" "$REF/impl/$app.c" -o "$OUT/${app}_dcamd" -L"$LIB" -ldcamd -Wl,-rpath,"$LIB" "$STDCXX" -lm
  echo "build_apps: built $OUT/${app}_ref $OUT/${app}_dcamd"
done
# the double apps: k-means / mm / lu use the double codecs and the MPI_Bcast_bitwise_* wrappers
# (libdcamd_mpi.so); their reference build needs the reference param.h next to the app
for app in k-means mm lu; do
  [ -f "$REF/impl/$app.c" ] || continue
  MPICH_CC=gcc "$MPI/bin/mpicc" -O3 -ffp-contract=off -w -iquote "$gen" -I- -I"$gen" -I"$REF/impl" \
      "$REF/impl/$app.c" "$REF/impl/dataCompression.c" -o "$OUT/${app}_ref" -lz -lm || { echo "build_apps: $app (reference build) failed"; continue; }
  MPICH_CC=gcc "$MPI/bin/mpicc" -O3 -w -DabsErrorBound="$BOUND" -iquote "$REPO/include" -I- -I"$REPO/include" \
      -I"$REF/impl" "$REF/impl/$app.c" -o "$OUT/${app}_dcamd" -L"$LIB" -ldcamd_mpi -ldcamd -Wl,-rpath,"$LIB" "$STDCXX" -lm \
      || { echo "build_apps: $app (libdcamd build) failed"; continue; }
  echo "build_apps: built $OUT/${app}_ref $OUT/${app}_dcamd"
done
