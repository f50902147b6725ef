#!/bin/bash
# One parametrised GPU-box batch (replaces the round-3 one-shot batch_r03*.sh scripts).
# From the repo root on the GPU box:
#   bash tools/gpu_batch.sh <out_dir> <step> [<step> ...]
# Steps (run in order; the batch stops at the first failing step):
#   probe                 host CPU facts (cpu_count, affinity, cgroup quota) -> <out>/probe.txt
#   tests[:<-k expr>]     pytest -m gpu (optionally -k; "+" stands for " or ") -> <out>/tests.log
#   alttests:<lib>:<-k expr>  the same -k subset against another build of the library (ab/<lib>.so)
#   envtests:<VAR=val>:<-k expr>  the same -k subset with one extra environment variable
#   smoke                 __graft_entry__.smoke() -> <out>/smoke.log
#   fuzz:<n>:<start>[:<filter>]  tools/debug/fuzz_campaign.py over seeds [start, start + n) -> <out>/fuzz_<filter>.txt
#   bench:<cfg>[:<tag>][:<args,comma,separated>]
#                         bench.py --config <cfg> --cpu-sample 0 [args] -> <out>/<cfg>_<tag>.json
#   abbench:<lib>:<cfg>:<tag>  the same against KCMC_LIB_PATH=<lib> (tools/ab_build.py) -> <out>/<cfg>_<tag>.json
#   envbench:<VAR=val>:<cfg>:<tag>[:<args,comma>]  the same with one extra environment variable
#   cpubench:<cfg>        bench.py --config <cfg> with its CPU baseline -> <out>/<cfg>_cpu.json
#   profile:<cfg>         tools/profile_round.sh (bench + rocprofv3 summary + warp PMC) -> <out>/<cfg>/
#   abpmc:<lib>:<cfg>:<tag>  the warp PMC passes (tools/pmc_warp.sh) against another build -> <out>/pmc_<tag>/
#   envtrace:<VAR=val>:<cfg>:<tag>  the same with one extra environment variable
#   trace:<cfg>:<tag>[:<args,comma>]  rocprofv3 --kernel-trace --memory-copy-trace of a short bench
#                         -> <out>/trace_<tag>/ (read with tools/timeline.py)
#   rehearse:<cfg>:<ranks>  bench.py over gloo ranks that share cuda:0 (the multi-rank path on one GPU)
#   lab:<binary>[:<tag>][:<args,comma,separated>]  a lab binary (tools/ or ab/) -> <out>/lab_<tag>.txt
#   envlab:<VAR=val>:<binary>:<tag>[:<args,comma>]  the same with one extra environment variable
#   labprof:<binary>:<tag>  a lab under rocprofv3 --kernel-trace --stats -> <out>/labprof_<tag>/
set -u
OUT=${1:?out dir}
shift
mkdir -p "$OUT"
for step in "$@"; do
  IFS=: read -r kind a b c d <<< "$step"
  case "$kind" in
    probe)
      { python -c "import os; print('cpu_count', os.cpu_count()); print('affinity', len(os.sched_getaffinity(0)))"
        cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cgroup v2 cpu.max"
        nproc; free -g | head -2; } > "$OUT/probe.txt" 2>&1
      cat "$OUT/probe.txt" ;;
    tests)
      K=()
      [ -n "${a:-}" ] && K=(-k "${a//+/ or }")  # tests:a+b = -k "a or b"
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" \
        > "$OUT/tests.log" 2>&1
      rc=$?
      echo "tests rc=$rc" >> "$OUT/tests.log"; tail -3 "$OUT/tests.log"
      [ $rc -eq 0 ] || exit 1 ;;
    alttests)  # alttests:<ab/lib.so>:<-k expr>  pytest -m gpu -k <expr> against another build (e.g. the sentinel one)
      KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH="$a" timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread -k "${b//+/ or }" > "$OUT/tests_alt.log" 2>&1
      rc=$?
      echo "alttests $a rc=$rc" >> "$OUT/tests_alt.log"; tail -3 "$OUT/tests_alt.log"
      [ $rc -eq 0 ] || exit 1 ;;
    envtests)  # envtests:<VAR=value>:<-k expr>  pytest -m gpu -k <expr> with one extra environment variable
      env "$a" timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${b//+/ or }" \
        > "$OUT/tests_env.log" 2>&1
      rc=$?
      echo "envtests $a rc=$rc" >> "$OUT/tests_env.log"; tail -3 "$OUT/tests_env.log"
      [ $rc -eq 0 ] || exit 1 ;;
    fuzz)
      timeout -k 10 900 python -u tools/debug/fuzz_campaign.py "$a" "$b" "${c:-}" > "$OUT/fuzz_${c:-all}.txt" 2>&1
      rc=$?
      grep -E "ok in|total" "$OUT/fuzz_${c:-all}.txt"
      [ $rc -eq 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
      tail -1 "$OUT/smoke.log" ;;
    bench)
      tag=${b:-1}
      IFS=, read -r -a X <<< "${c:-}"
      timeout -k 10 300 python bench.py --config "$a" --cpu-sample 0 "${X[@]}" > "$OUT/${a}_$tag.json" \
        2>> "$OUT/bench.err" || exit 1
      echo "$a $tag: $(head -c 160 "$OUT/${a}_$tag.json")" ;;
    abbench)  # abbench:<ab/lib.so>:<cfg>:<tag>  the bench against another build of the library
      KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH="$a" timeout -k 10 300 python bench.py --config "$b" --cpu-sample 0 > "$OUT/${b}_$c.json" \
        2>> "$OUT/bench.err" || exit 1
      echo "$b $c ($a): $(head -c 160 "$OUT/${b}_$c.json")" ;;
    envbench)  # envbench:<VAR=value>:<cfg>:<tag>[:<args,comma>]  the bench with one extra environment variable
      IFS=, read -r -a X <<< "${d:-}"
      env "$a" timeout -k 10 300 python bench.py --config "$b" --cpu-sample 0 "${X[@]}" > "$OUT/${b}_$c.json" \
        2>> "$OUT/bench.err" || exit 1
      echo "$b $c ($a): $(head -c 160 "$OUT/${b}_$c.json")" ;;
    cpubench)
      timeout -k 10 400 python bench.py --config "$a" > "$OUT/${a}_cpu.json" 2>> "$OUT/bench.err" || exit 1
      echo "$a cpu: $(head -c 160 "$OUT/${a}_cpu.json")" ;;
    profile)
      bash tools/profile_round.sh "$OUT/$a" --config "$a" || exit 1 ;;
    abpmc)
      KCMC_TEST_ONLY_ALT_LIB=1 KCMC_LIB_PATH="$a" bash tools/pmc_warp.sh "$OUT/pmc_$c" "warp_affine_u16|warp_perspective_u16" --config "$b" \
        || exit 1 ;;
    trace)
      IFS=, read -r -a X <<< "${c:-}"
      R=$PWD
      (cd /tmp && export TMPDIR=/tmp && cd "$R" &&
        timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/$OUT/trace_$b" \
          -o run -- python bench.py --config "$a" --cpu-sample 0 --steps 12 --warmup 3 "${X[@]}" \
          > "$OUT/trace_$b.json" 2> "$OUT/trace_$b.err") || exit 1
      echo "trace $a $b: $(head -c 160 "$OUT/trace_$b.json")" ;;
    envtrace)  # envtrace:<VAR=value[+VAR=value]>:<cfg>:<tag>  the trace step with extra environment variables
      R=$PWD
      IFS=+ read -r -a E <<< "$a"
      (cd /tmp && export TMPDIR=/tmp && cd "$R" &&
        env "${E[@]}" timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/$OUT/trace_$c" \
          -o run -- python bench.py --config "$b" --cpu-sample 0 --steps 12 --warmup 3 \
          > "$OUT/trace_$c.json" 2> "$OUT/trace_$c.err") || exit 1
      echo "trace $b $c ($a): $(head -c 160 "$OUT/trace_$c.json")" ;;
    envlab)  # envlab:<VAR=value>:<binary>:<tag>[:<args,comma>]  a lab with one extra environment variable
      IFS=, read -r -a X <<< "${d:-}"
      env "$a" timeout -k 10 240 "$b" "${X[@]}" > "$OUT/lab_$c.txt" 2>&1 || exit 1
      tail -4 "$OUT/lab_$c.txt" ;;
    rehearse)  # rehearse:<cfg>:<ranks>  bench.py over <ranks> gloo ranks sharing cuda:0 (the N>1 code path)
      KCMC_BENCH_BACKEND=gloo KCMC_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$b" --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus "$b" --steps 5 --warmup 2 \
        --config "$a" --cpu-sample 0 > "$OUT/rehearse_${a}_$b.json" 2>> "$OUT/rehearse.err" || exit 1
      echo "rehearse $a x$b: $(tail -1 "$OUT/rehearse_${a}_$b.json" | head -c 200)" ;;
    labprof)  # labprof:<binary>:<tag>  a lab under rocprofv3 --kernel-trace --stats -> <out>/labprof_<tag>/
      R=$PWD
      (cd /tmp && export TMPDIR=/tmp && cd "$R" &&
        timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/labprof_$b" -o run \
          -- "$a" > "$OUT/labprof_$b.txt" 2>&1) || exit 1
      tail -2 "$OUT/labprof_$b.txt" ;;
    lab)
      tag=${b:-$(basename "$a")}
      IFS=, read -r -a X <<< "${c:-}"
      timeout -k 10 240 "$a" "${X[@]}" > "$OUT/lab_$tag.txt" 2>&1 || exit 1
      tail -4 "$OUT/lab_$tag.txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
