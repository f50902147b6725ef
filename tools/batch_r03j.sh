#!/bin/bash
# Round-3 batch 10 (from the repo root):  bash tools/batch_r03j.sh <out>
# depth-2 match beside as the c2 / c3 default: sharded + pipeline GPU tests, c2 / c3 at the
# new defaults, c4 at depth 2 beside against its depth-3 default, one round each + c2/c3 twice
set -u
OUT=${1:-gpurun_out/r03_batch10}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "pipeline or sharded" > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for r in 1 2; do
  for c in c2 c3; do
    timeout -k 10 240 python bench.py --config $c --cpu-sample 0 > "$OUT/${c}_$r.json" 2>> "$OUT/bench.err" || exit 1
  done
done
timeout -k 10 240 python bench.py --config c4 --cpu-sample 0 > "$OUT/c4_d3b.json" 2>> "$OUT/bench.err" || exit 1
timeout -k 10 240 python bench.py --config c4 --cpu-sample 0 --pipeline-depth 2 > "$OUT/c4_d2b.json" 2>> "$OUT/bench.err" || exit 1
echo done
