#!/bin/bash
# Same-box A/B of warp lab builds (tools/warp_lab.hip in LAB_LIB mode: the library's
# configuration, 3 repeats per data set + output checksum), two rounds over the builds:
#   bash tools/warp_ab.sh <out_dir> <lab> [<lab> ...]      (FRAMES, LAB_DIST from the env)
set -u
OUT=$1; shift
F=${FRAMES:-2000}
mkdir -p "$OUT"
python tools/write_texture.py "$OUT/tex.u16" || exit 1
for r in 1 2; do
  for L in "$@"; do
    echo "== $(basename "$L") (round $r)" >> "$OUT/ab.txt"
    LAB_LIB=1 timeout -k 10 120 "$L" "$F" "$OUT/tex.u16" >> "$OUT/ab.txt" 2>&1 || exit 1
  done
done
rm -f "$OUT/tex.u16"
