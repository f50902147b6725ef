#!/bin/bash
# PMC passes for the dominant kernel (warp) of bench.py, one rocprofv3 run per counter
# group (rocprofv3 does not split counters over passes).  Run on the GPU box from the
# repo root:  bash tools/pmc_warp.sh <out_dir> [kernel_regex] [bench args...]
set -u
OUT=${1:-gpurun_out/pmc}
RE=${2:-warp_affine}
shift $(( $# < 2 ? $# : 2 ))
EXTRA=("$@")
R=$PWD
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$R"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RE" --pmc "$@" --output-format csv \
    -d "$R/$OUT/$name" -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample 0 "${EXTRA[@]}" \
    > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU && \
run sq2 GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
