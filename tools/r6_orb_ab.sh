# round 6: same-box A/B of ORB detector builds in ab/ (tools/orb_rates.py), interleaved,
# two rounds, after the in-tree build's detector tests and an orb fuzz campaign
set -u
O=${1:-gpurun_out/r06_o}
shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_pipeline.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "orb or detect" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 python -u tools/debug/fuzz_campaign.py 1000 80000 orb > $O/fuzz_orb.txt 2>&1 || { tail -20 $O/fuzz_orb.txt; exit 1; }
grep -E "ok in|total" $O/fuzz_orb.txt
for round in 1 2; do
  for l in "$@"; do
    KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=ab/$l.so timeout -k 10 200 python tools/orb_rates.py >> $O/rates.txt \
      2>> $O/rates.err || exit 1
  done
done
cat $O/rates.txt
