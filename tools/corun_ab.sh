mkdir -p gpurun_out/h3
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/h3/tests.log 2>&1 || { tail -30 gpurun_out/h3/tests.log; exit 1; }
tail -1 gpurun_out/h3/tests.log
for cfg in c2 c3 c5; do for r in 1 2; do for c in 0 1 2; do
  timeout -k 10 200 python bench.py --cpu-sample 0 --config $cfg --corun $c > gpurun_out/h3/b.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/h3/b.json'));print('$cfg corun $c', d['value'],d['ms_per_step'],d['stage_ms']['warp'])"
done; done; done
