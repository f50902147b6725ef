#!/bin/bash
# Round-3 batch 8 (from the repo root):  bash tools/batch_r03h.sh <out>
# hand-written top-6 step of the float matcher: its GPU tests, then c5 twice
set -u
OUT=${1:-gpurun_out/r03_batch8}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "f32 or configs or models" > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for r in 1 2; do
  timeout -k 10 240 python bench.py --config c5 --cpu-sample 0 > "$OUT/c5_$r.json" 2>> "$OUT/bench.err" || exit 1
done
echo done
