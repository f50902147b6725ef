#!/bin/bash
# Builds ablations / variants of the float matcher (match_f32.hip) for tools/knn_lab.hip
# -DKNN_F32 into ab/ (run here, on the CPU):
#   base   match_f32.hip as it is
#   (a timing-only variant without the top-K insertion decodes garbage keys into row ids
#    and faults the epilogue: not built any more)
#   k5     a top-5 instead of the top-6 per lane
# then on the box:  for v in base k5; do ab/knnf_lab_$v; done
set -eu
MF32=keypoint-consensus-motion-correction_amd/csrc/match_f32.hip
mkdir -p ab
grep -q "constexpr int kTop = 6; " $MF32
cp $MF32 ab/matchf_base.hip
sed "s/constexpr int kTop = 6; /constexpr int kTop = 5; /" $MF32 > ab/matchf_k5.hip
VARS=${VARS:-base k5}
for v in $VARS; do
  ! cmp -s $MF32 ab/matchf_$v.hip || [ $v = base ] || { echo "f32 edit for $v did not apply"; exit 1; }
  sed -i 's|#include "kcmc_internal.h"|#include "../keypoint-consensus-motion-correction_amd/csrc/kcmc_internal.h"|' ab/matchf_$v.hip
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -DKNN_F32 -DMATCH_SRC="\"../ab/matchf_$v.hip\"" \
    tools/knn_lab.hip -o ab/knnf_lab_$v &
done
wait
ls -la ab/knnf_lab_*
