#!/bin/bash
# Same-box A/B of RANSAC library builds (tools/ransac_rates.py), two rounds:
#   bash tools/ransac_ab.sh <config> ab/<a>.so ab/<b>.so ...
set -u
C=$1; shift
for r in 1 2; do
  for L in "$@"; do
    KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=$L timeout -k 10 120 python tools/ransac_rates.py --config "$C" || exit 1
  done
done
