#!/bin/bash
# Same-box A/B of warp lab builds (tools/warp_lab.hip in LAB_LIB mode: the library's
# configuration, 3 repeats per data set + output checksum), alternating the builds:
#   bash tools/warp_ab.sh <out_dir> <lab_a> <lab_b> [frames]
set -u
OUT=$1; A=$2; B=$3; F=${4:-2000}
mkdir -p "$OUT"
python tools/write_texture.py "$OUT/tex.u16" || exit 1
for r in 1 2; do
  for L in "$A" "$B"; do
    echo "== $(basename "$L") (round $r)" >> "$OUT/ab.txt"
    LAB_LIB=1 timeout -k 10 120 "$L" "$F" "$OUT/tex.u16" >> "$OUT/ab.txt" 2>&1 || exit 1
  done
done
rm -f "$OUT/tex.u16"
