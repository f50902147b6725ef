# round 6: the drop-in split (bench.py --single-process --devices 0) with the device-map warp
# (default) against the warp behind the host post-processing (chain_probe hostmaps), same
# box, interleaved; the multidevice GPU tests first
set -u
O=${1:-gpurun_out/r06_s}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multidevice.py tests/test_gpu_pipeline.py -x -q --timeout 120 \
  --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for c in ${R6_CONFIGS:-c3 c2}; do
  for v in none hostmaps none hostmaps; do
    echo "== $c $v" >> $O/lines.txt
    timeout -k 10 240 python tools/chain_probe.py $v -- --config $c --single-process --devices 0 --steps 40 \
      --warmup 5 --cpu-sample 0 >> $O/lines.txt 2>> $O/err.txt || exit 1
  done
done
python - $O/lines.txt <<'EOF'
import json, sys
v = None
for l in open(sys.argv[1]):
    if l.startswith("=="):
        v = l[3:].strip()
    elif l.startswith("{"):
        d = json.loads(l)
        print(f"{v:16s} {d['value']:12.0f} frames/s  {d['ms_per_step']:.3f} ms")
EOF
