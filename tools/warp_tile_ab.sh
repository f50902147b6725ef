#!/bin/bash
# Same-box A/B of two library builds (tools/ab_build.py) on the c3 and c2 benches, two
# rounds, after the warp GPU tests against the variant:  bash tools/warp_tile_ab.sh <out> <base.so> <var.so>
set -u
OUT=$1; B=$2; V=$3
mkdir -p "$OUT"
KCMC_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "warp" > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for r in 1 2; do
  for L in $B $V; do
    n=$(basename $L .so)
    for c in c3 c2; do
      KCMC_LIB_PATH=$L timeout -k 10 240 python bench.py --config $c --cpu-sample 0 > "$OUT/${c}_${n}_$r.json" 2>> "$OUT/bench.err" || exit 1
    done
  done
done
echo done
