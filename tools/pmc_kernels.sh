#!/bin/bash
# PMC passes for the analysis kernels of bench.py (K1 match, K2 RANSAC): VALU / MFMA /
# FP64 instruction counts and busy cycles, one rocprofv3 run per pass (rocprofv3 does
# not split counters over passes; <= 8 SQ + 2 GRBM counters each).  Counters missing
# from `rocprofv3 -L` on this box are dropped from their pass.  Run on the GPU box from
# the repo root:   bash tools/pmc_kernels.sh <out_dir> [kernel_regex] [bench args...]
# (PMC_CMD="python tools/match_rates.py --configs c4" profiles that command instead)
# then:            python tools/pmc_summary.py <out_dir> --by-kernel --json <out>.json
set -u
OUT=${1:-gpurun_out/pmck}
RE=${2:-knn2|ransac|match_filter}
shift $(( $# < 2 ? $# : 2 ))
EXTRA=("$@")
R=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
have() {  # keep the counters this box lists
  local keep=()
  for c in "$@"; do grep -qw "$c" "$OUT/counters.txt" && keep+=("$c"); done
  echo "${keep[@]}"
}
run() {  # name, counters...
  local name=$1; shift
  local ctr
  ctr=$(have "$@")
  [ -z "$ctr" ] && { echo "pass $name: no counters"; return 0; }
  echo "pass $name: $ctr"
  # shellcheck disable=SC2086
  if [ -n "${PMC_CMD:-}" ]; then
    # shellcheck disable=SC2086
    timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RE" --pmc $ctr --output-format csv \
      -d "$R/$OUT/$name" -o run -- $PMC_CMD > "$OUT/$name.json" 2> "$OUT/$name.err"
  else
    timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RE" --pmc $ctr --output-format csv \
      -d "$R/$OUT/$name" -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 --serial "${EXTRA[@]}" \
      > "$OUT/$name.json" 2> "$OUT/$name.err"
  fi
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run valu GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY && \
run mfma GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
run lds GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES && \
run f64 GRBM_GUI_ACTIVE SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32
