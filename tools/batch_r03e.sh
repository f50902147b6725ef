#!/bin/bash
# Round-3 batch 5 (from the repo root):  bash tools/batch_r03e.sh <out>
# c4 schedules: the match beside the warp (depth 3) against the default (depth 2, match
# then warp on the kernel stream), two rounds each.
set -u
OUT=${1:-gpurun_out/r03_batch5}
mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 240 python bench.py --config c4 --cpu-sample 0 > "$OUT/c4_$r.json" 2>> "$OUT/bench.err" || exit 1
  timeout -k 10 240 python bench.py --config c4 --cpu-sample 0 --pipeline-depth 3 --match-beside > "$OUT/c4_beside_$r.json" 2>> "$OUT/bench.err" || exit 1
  timeout -k 10 240 python bench.py --config c4 --cpu-sample 0 --pipeline-depth 3 > "$OUT/c4_d3_$r.json" 2>> "$OUT/bench.err" || exit 1
done
echo done
