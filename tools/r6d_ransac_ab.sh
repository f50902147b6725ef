# round 6: same-box A/B of the RANSAC scorers (tools/ransac_rates.py) over library builds in ab/
set -u
O=${1:-gpurun_out/r06_e}
shift
mkdir -p $O
for c in ${R6_CONFIGS:-c3 c2}; do
  for l in "$@"; do
    KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=ab/$l.so timeout -k 10 120 python tools/ransac_rates.py --config $c --reps 15 >> $O/rates.txt 2>> $O/rates.err || exit 1
  done
done
cat $O/rates.txt
