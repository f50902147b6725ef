#!/bin/bash
# Round-3 batch 6 (from the repo root):  bash tools/batch_r03f.sh <out>
# the float matcher at 6 waves per SIMD: its GPU tests, then c5 twice and c4 at its new
# default schedule (match beside the warp)
set -u
OUT=${1:-gpurun_out/r03_batch6}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "f32 or models or configs or pipeline" > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for r in 1 2; do
  timeout -k 10 240 python bench.py --config c5 --cpu-sample 0 > "$OUT/c5_$r.json" 2>> "$OUT/bench.err" || exit 1
done
timeout -k 10 240 python bench.py --config c4 --cpu-sample 0 > "$OUT/c4.json" 2>> "$OUT/bench.err" || exit 1
echo done
