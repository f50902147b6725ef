#!/bin/bash
# Same-box A/B of u8 matcher lab builds (tools/knn_lab.hip): two rounds over the builds at
# the c4 / c3 / c2 shapes.   bash tools/knn_ab.sh <out_dir> <lab> [<lab> ...]
set -u
OUT=$1; shift
mkdir -p "$OUT"
for r in 1 2; do
  for L in "$@"; do
    for shape in "4096 61 625 4506" "500 61 2500 550" "500 32 2000 550"; do
      echo "== $(basename "$L") $shape (round $r)" >> "$OUT/ab.txt"
      # shellcheck disable=SC2086
      timeout -k 10 60 "$L" $shape 20 >> "$OUT/ab.txt" 2>&1 || exit 1
    done
  done
done
