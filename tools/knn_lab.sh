#!/bin/bash
# Builds the K1 u8 matcher ablations of tools/knn_lab.hip into ab/ (run here, on the CPU):
#   base   match.hip as it is
#   nomfma the MFMAs replaced by one VALU op per k-step (epilogue on near-constant keys)
# then on the box:  for v in base nomfma; do ab/knn_lab_$v; done; for v in base noepi nomfma; do ab/knnf_lab_$v; done
# (an ablation that removes most of the compute also exposes the staged chunk's load
# latency, so the differences are not cost shares)
set -eu
M=keypoint-consensus-motion-correction_amd/csrc/match.hip
mkdir -p ab
MF='acc\[b\] = __builtin_amdgcn_mfma_i32_32x32x32_i8(afrag\[kk\], bfrag\[b\]\[kk\], acc\[b\], 0, 0, 0);'
grep -q "__builtin_amdgcn_mfma_i32_32x32x32_i8(afrag\[kk\]" $M
cp $M ab/match_base.hip
sed "s/$MF/acc[b][kk] += afrag[kk][0] ^ bfrag[b][kk][0];/" $M > ab/match_nomfma.hip
for v in base nomfma; do
  ! cmp -s $M ab/match_$v.hip || [ $v = base ] || { echo "edit for $v did not apply"; exit 1; }
  sed -i 's|#include "kcmc_internal.h"|#include "../keypoint-consensus-motion-correction_amd/csrc/kcmc_internal.h"|' ab/match_$v.hip
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -DMATCH_SRC="\"../ab/match_$v.hip\"" \
    tools/knn_lab.hip -o ab/knn_lab_$v &
done
wait
# float matcher (match_f32.hip, -DKNN_F32): base / noepi (top-4 epilogue replaced by one
# XOR) / nomfma (the three bf16 MFMAs replaced by one VALU op)
MF32=keypoint-consensus-motion-correction_amd/csrc/match_f32.hip
E32='top4_key(ck\[b\], ok ? ((xb \& ~63u) | (uint32_t)row) : kNoKey);'
grep -q "top4_key(ck\[b\], ok ?" $MF32
cp $MF32 ab/matchf_base.hip
sed "s/$E32/{ if (r == 0) ck[b][0] ^= xb; }/" $MF32 > ab/matchf_noepi.hip
sed -e 's/acc\[b\] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, bhi\[b\]\[st\], acc\[b\], 0, 0, 0);/acc[b][st] += (float)a_h[0] * (float)bhi[b][st][0];/' \
    -e '/__builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, blo/d' -e '/__builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l, bhi/d' $MF32 > ab/matchf_nomfma.hip
for v in base noepi nomfma; do
  ! cmp -s $MF32 ab/matchf_$v.hip || [ $v = base ] || { echo "f32 edit for $v did not apply"; exit 1; }
  sed -i 's|#include "kcmc_internal.h"|#include "../keypoint-consensus-motion-correction_amd/csrc/kcmc_internal.h"|' ab/matchf_$v.hip
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -DKNN_F32 -DMATCH_SRC="\"../ab/matchf_$v.hip\"" \
    tools/knn_lab.hip -o ab/knnf_lab_$v &
done
wait
ls -la ab/knnf_lab_*
