#!/bin/bash
# The measurement set behind a round's bench line, on the GPU box, from the repo root:
#   bash tools/profile_round.sh <out_dir> [bench args...]
# 1. bench.py (default: c2 with the CPU baseline) -> <out>/bench.json
# 2. rocprofv3 --kernel-trace --stats of the same bench command (no CPU baseline)
#    -> <out>/prof/run_kernel_stats.csv
# 3. the warp's PMC passes (tools/pmc_warp.sh: HBM bytes, instruction mix) -> <out>/pmc
# Then, in the build container: python tools/collect_profiles.py <out> <tag>, which files
# them under profiles/ with the commit they were measured on.
set -u
OUT=${1:-gpurun_out/round}
shift $(( $# < 1 ? $# : 1 ))
R=$PWD
mkdir -p "$OUT"
timeout -k 10 300 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
echo "bench: $(head -c 300 "$OUT/bench.json")"
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o run -- \
  python bench.py --cpu-sample 0 "$@" > "$OUT/bench_under_rocprof.json" 2> "$OUT/prof.err" || exit 1
echo "rocprofv3 kernel trace: done"
bash tools/pmc_warp.sh "$OUT/pmc" "warp_affine_u16|warp_perspective_u16" "$@"
