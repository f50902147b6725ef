#!/bin/bash
# Same-box A/B of the two schedules of OverlappedSlabs (RANSAC beside the warp, the
# default, vs behind it on the kernel stream) on c2 / c3 / c5, two rounds each:
#   bash tools/corun_ab.sh [out_dir]
# (the round-2 A/B also ran a third variant with the match beside the warp, since
# removed: DESIGN.md section 6)
set -u
OUT=${1:-gpurun_out/corun_ab}
mkdir -p "$OUT"
for cfg in c2 c3 c5; do for r in 1 2; do for v in "" "--no-corun"; do
  timeout -k 10 200 python bench.py --cpu-sample 0 --config $cfg $v > "$OUT/b.json" || exit 1
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$cfg ${v:-corun}', d['value'], d['ms_per_step'], d['stage_ms']['warp'])"
done; done; done
