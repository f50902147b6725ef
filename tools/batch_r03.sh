#!/bin/bash
# Round-3 measurement batch on the GPU box (from the repo root):  bash tools/batch_r03.sh <out>
# GPU tests, float-matcher lab A/B, c3 schedule A/B (three-slab default vs match beside the
# warp), a c3 kernel trace of the match-beside schedule, and the 2-rank gloo rehearsal.
set -u
OUT=${1:-gpurun_out/r03_batch}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/tests.log"; tail -2 "$OUT/tests.log"
grep -q "tests rc=0" "$OUT/tests.log" || exit 1
for v in ${LAB_VARS:-fb2 br2 fb2 br2}; do
  timeout -k 10 60 ab/knnf_lab_$v >> "$OUT/lab.txt" 2>&1 || exit 1; echo "^ $v" >> "$OUT/lab.txt"
done
for r in 1 2; do
  for m in "" "--match-beside"; do
    timeout -k 10 200 python bench.py --config c3 --cpu-sample 0 $m > "$OUT/c3${m:+_beside}_$r.json" 2>> "$OUT/bench.err" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$PWD/$OUT/prof_c3_beside" -o run -- \
  python bench.py --config c3 --cpu-sample 0 --steps 20 --match-beside > "$OUT/c3_beside_prof.json" 2>> "$OUT/bench.err" || exit 1
for c in c3 c2; do
  KCMC_BENCH_BACKEND=gloo KCMC_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --config $c --cpu-sample 0 \
    > "$OUT/rehearsal_2ranks_$c.json" 2>> "$OUT/rehearsal.err" || exit 1
done
echo done
