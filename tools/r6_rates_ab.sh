# round 6: same-box A/B of RANSAC library builds in ab/ with the pipelines' device lists
# (tools/ransac_rates.py --device-lists), interleaved, two rounds; one JSON line per run
set -u
O=${1:-gpurun_out/r06_r}
shift
mkdir -p $O
for round in 1 2; do
  for c in ${R6_CONFIGS:-c2}; do
    for l in "$@"; do
      KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH=ab/$l.so timeout -k 10 120 python tools/ransac_rates.py --config $c \
        --reps 21 --device-lists >> $O/rates.txt 2>> $O/rates.err || exit 1
    done
  done
done
python - $O/rates.txt <<'EOF'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['config']}  {d['lib']:18s} median {d['ms_median']:.4f} ms  best {d['ms_best']:.4f}  digest {d['digest']}")
EOF
