#!/bin/bash
# Round-3 batch 4 (from the repo root):  bash tools/batch_r03d.sh <out>
set -u
OUT=${1:-gpurun_out/r03_batch4}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pipeline or sharded" > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --config c3 --cpu-sample 0 > "$OUT/c3_$r.json" 2>> "$OUT/bench.err" || exit 1
  timeout -k 10 200 python bench.py --config c3 --cpu-sample 0 --fit-after-warp > "$OUT/c3_late_$r.json" 2>> "$OUT/bench.err" || exit 1
done
timeout -k 10 200 python bench.py --config c5 --cpu-sample 0 --pipeline-depth 3 > "$OUT/c5_d3.json" 2>> "$OUT/bench.err" || exit 1
timeout -k 10 200 python bench.py --config c2 --cpu-sample 0 --pipeline-depth 3 > "$OUT/c2_d3.json" 2>> "$OUT/bench.err" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$PWD/$OUT/prof_c3" -o run -- \
  python bench.py --config c3 --cpu-sample 0 --steps 20 > "$OUT/c3_prof.json" 2>> "$OUT/bench.err" || exit 1
echo done
