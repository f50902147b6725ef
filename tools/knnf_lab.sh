#!/bin/bash
# Builds variants of the float matcher (match_f32.hip) for tools/knn_lab.hip -DKNN_F32
# into ab/ (run here, on the CPU), one per value of a compile-time knob:
#   KNOB=KCMC_IMG_ROWS VALS="1 2 4 8"   (frame_images_kernel rows per 16-lane group)
# then on the box:  ab/knnf_lab_<KNOB>_<val> for each value.
set -eu
KNOB=${KNOB:-KCMC_IMG_ROWS}
VALS=${VALS:-1 4}
mkdir -p ab
for v in $VALS; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -DKNN_F32 -D$KNOB=$v \
    tools/knn_lab.hip -o ab/knnf_lab_${KNOB}_$v &
done
wait
ls -la ab/knnf_lab_*
