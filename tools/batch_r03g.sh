#!/bin/bash
# Round-3 batch 7 (from the repo root):  bash tools/batch_r03g.sh <out>
# lookup_order with LDS-staged keys: consensus / pipeline GPU tests, then c3 and c2 twice
set -u
OUT=${1:-gpurun_out/r03_batch7}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "consensus or pipeline or sharded or configs" > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for r in 1 2; do
  timeout -k 10 240 python bench.py --config c3 --cpu-sample 0 > "$OUT/c3_$r.json" 2>> "$OUT/bench.err" || exit 1
  timeout -k 10 240 python bench.py --config c2 --cpu-sample 0 > "$OUT/c2_$r.json" 2>> "$OUT/bench.err" || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_c3" -o run -- \
  python bench.py --config c3 --cpu-sample 0 --steps 20 > "$OUT/c3_prof.json" 2>> "$OUT/bench.err" || exit 1
echo done
