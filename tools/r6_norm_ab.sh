# round 6: same-box A/B of the normalisation builds in ab/ (tools/norm_rates.py), interleaved,
# two rounds, after the normalisation tests and a pyr_norm fuzz campaign on the in-tree build
set -u
O=${1:-gpurun_out/r06_h}
shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "percentile or brightest or max_scale or normal or pyr" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 python -u tools/debug/fuzz_campaign.py 1000 81000 pyr_norm > $O/fuzz_pyr_norm.txt 2>&1 || { tail -20 $O/fuzz_pyr_norm.txt; exit 1; }
grep -E "ok in|total" $O/fuzz_pyr_norm.txt
for round in 1 2; do
  for l in "$@"; do
    KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=ab/$l.so timeout -k 10 200 python tools/norm_rates.py >> $O/rates.txt \
      2>> $O/rates.err || exit 1
  done
done
cat $O/rates.txt
