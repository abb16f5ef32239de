timeout -k 10 400 python -u -m pytest tests/test_fast_mode.py -m gpu -k "seg" -x -q --timeout 120 --timeout-method thread > gpurun_out/r6g_seg_tests.log 2>&1; tail -2 gpurun_out/r6g_seg_tests.log
for w in 2 3 4; do
  B2H_SEG_WAVES=$w timeout -k 10 300 python -u bench.py --lz-mode seg --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r6g_seg_bench_w$w.log 2>&1 || { echo "bench w$w failed"; tail -5 gpurun_out/r6g_seg_bench_w$w.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6g_seg_bench_w$w.log').read().strip().splitlines()[-1]); print('W=$w', d['value'], d['modes'])"
done
