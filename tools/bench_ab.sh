#!/bin/bash
# Same-box A/B of bench.py variants, two rounds; each argument is one variant, given as
# "<lib or -> <bench args...>" (lib: an ab/ build for KCMC_LIB_PATH, - for the in-tree one):
#   bash tools/bench_ab.sh <out_dir> "- --no-corun" "ab/x.so" ...
set -u
OUT=$1; shift
mkdir -p "$OUT"
VARIANTS=("$@")
for r in 1 2; do
  for v in "${VARIANTS[@]}"; do
    read -r L ARGS <<< "$v"
    if [ "$L" = "-" ]; then unset KCMC_LIB_PATH; else export KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=$L; fi
    # shellcheck disable=SC2086
    timeout -k 10 200 python bench.py --cpu-sample 0 $ARGS > "$OUT/b.json" || exit 1
    python -c "import json,sys;d=json.load(open('$OUT/b.json'));print('$v', d['value'], d['ms_per_step'], d['stage_ms']['warp'], d['stage_ms']['match'])"
  done
done
