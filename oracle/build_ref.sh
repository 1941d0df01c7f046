#!/usr/bin/env bash
# Builds the reference's three MPI executables from their own sources, where they lie under
# /root/reference/src, into oracle/_ref/ (git-ignored; never copied into the repo).
# Same command line as the reference's test.sh:10 (mpicc <alg>.c matr_utils.c utils.c -Wall -lm,
# no -O), plus -include oracle/ref_dump.h so rank 0 dumps y. Needs the image's MPICH
# (/opt/conda/bin/mpicc; its wrapper's default compiler is absent, so MPICH_CC=gcc).
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF="${REF:-/root/reference}"
MPICC="${MPICC:-/opt/conda/bin/mpicc}"
OUT="$HERE/_ref"
if [ ! -d "$REF/src" ]; then echo "build_ref: $REF/src not present, skipping"; exit 0; fi
if [ ! -x "$MPICC" ]; then echo "build_ref: $MPICC not present, skipping"; exit 0; fi
mkdir -p "$OUT"
for alg in rowwise colwise blockwise; do
  MPICH_CC=gcc "$MPICC" -include "$HERE/ref_dump.h" "$REF/src/multiplier_$alg.c" \
      "$REF/src/matr_utils.c" "$REF/src/utils.c" -o "$OUT/multiplier_$alg" -Wall -lm 2> "$OUT/build_$alg.log" \
      || { cat "$OUT/build_$alg.log"; exit 1; }
done
echo "build_ref: built $(ls "$OUT" | grep -c '^multiplier_') reference executables in $OUT"
