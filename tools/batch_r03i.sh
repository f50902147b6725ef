#!/bin/bash
# Round-3 batch 9 (from the repo root):  bash tools/batch_r03i.sh <out>
# depth-2 match beside the warp: pipeline GPU tests, then c2 / c3 / c5 against the
# defaults, two rounds
set -u
OUT=${1:-gpurun_out/r03_batch9}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pipeline" > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for r in 1 2; do
  for c in c2 c3 c5; do
    timeout -k 10 240 python bench.py --config $c --cpu-sample 0 > "$OUT/${c}_$r.json" 2>> "$OUT/bench.err" || exit 1
    timeout -k 10 240 python bench.py --config $c --cpu-sample 0 --pipeline-depth 2 --match-beside > "$OUT/${c}_b2_$r.json" 2>> "$OUT/bench.err" || exit 1
  done
done
echo done
