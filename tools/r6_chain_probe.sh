# round 6: upper bounds for the c3 analysis chain (tools/chain_probe.py), same box,
# interleaved; one bench line per variant in $O/lines.txt
set -u
O=${1:-gpurun_out/r06_p}
C=${2:-c3}
mkdir -p $O
for v in none lookup spin vote,lookup merge,vote,lookup none ransac match,vote,merge,lookup lookup spin none; do
  echo "== $v" >> $O/lines.txt
  timeout -k 10 240 python tools/chain_probe.py $v -- --config $C --steps 60 --warmup 5 --cpu-sample 0 \
    >> $O/lines.txt 2>> $O/err.txt || exit 1
done
cat $O/lines.txt
