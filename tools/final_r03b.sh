#!/bin/bash
# Round-3 closing measurement set (from the repo root):  bash tools/final_r03b.sh <out>
# GPU tests, smoke, tools/profile_round.sh at c2 and at c4 (bench line with the CPU
# baseline, rocprofv3 kernel summary, warp PMC passes), the c3 / c5 bench lines.
set -u
OUT=${1:-gpurun_out/r03_close2}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/gpu_tests.log"; tail -2 "$OUT/gpu_tests.log"
grep -q "tests rc=0" "$OUT/gpu_tests.log" || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
bash tools/profile_round.sh "$OUT/c2" || exit 1
bash tools/profile_round.sh "$OUT/c4" --config c4 || exit 1
for c in c3 c5; do
  mkdir -p "$OUT/$c"
  timeout -k 10 300 python bench.py --config $c > "$OUT/$c/bench.json" 2> "$OUT/$c/bench.err" || exit 1
done
echo done
