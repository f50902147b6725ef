#!/bin/bash
# The warp's LDS-sentinel debug build (warp.hip, KCMC_WARP_SENTINEL): every workgroup fills
# its whole LDS array with 0xFFFF before staging its box, so a tap read outside the staged
# rows / columns gives a deterministic wrong value instead of an earlier workgroup's data.
# Build here (CPU):   bash tools/debug/warp_sentinel.sh            -> ab/sentinel.so
# Run on the box:     bash tools/gpu_batch.sh <out> alttests:ab/sentinel.so:warp+config
set -eu
cd "$(dirname "$0")/../.."
KCMC_AB_FLAGS="-DKCMC_WARP_SENTINEL" python tools/ab_build.py sentinel
