#!/usr/bin/env bash
# Compile the reference codec library (impl/dataCompression.c, read in place from
# /root/reference) into oracle/_ref/libref_<bound>.so, one per absErrorBound.
# The reference selects the bound with a compile-time macro that impl/set-parameter.sh edits with
# sed; we do the same without touching the reference: a generated dataCompression.h in
# _ref/gen_<bound>/ includes the original header and redefines absErrorBound, and `-iquote ... -I-`
# makes the compiler pick it instead of the header next to dataCompression.c.
# Nothing is copied from the reference into the repository; outputs go to oracle/_ref/ only.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
MPI_INC=${MPI_INC:-/opt/conda/include}
MPI_LIB=${MPI_LIB:-/opt/conda/lib}
if [ ! -f "$REF/impl/dataCompression.c" ]; then
  echo "build_ref: $REF not present, skipping reference build"; exit 0
fi
mkdir -p "$OUT"
for b in 0.001 0.000001 0.0001 0.01; do
  tag=$(python3 -c "print('%g' % $b)")
  gen="$OUT/gen_$tag"
  mkdir -p "$gen"
  printf '#include "%s/impl/dataCompression.h"\n#undef absErrorBound\n#define absErrorBound %s\n' "$REF" "$b" > "$gen/dataCompression.h"
  lib="$OUT/libref_$tag.so"
  if [ ! -f "$lib" ] || [ "$REF/impl/dataCompression.c" -nt "$lib" ]; then
    gcc -O3 -ffp-contract=off -fPIC -shared -w -iquote "$gen" -I- -I"$gen" -I"$REF/impl" -I"$MPI_INC" \
        "$REF/impl/dataCompression.c" -o "$lib" -L"$MPI_LIB" -lmpi -lz -lm -Wl,-rpath,"$MPI_LIB" 2>/dev/null
    echo "build_ref: built $lib"
  fi
done
