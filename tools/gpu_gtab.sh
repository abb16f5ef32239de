# Hash table in LDS vs in global memory: encoder micro-benchmark on planes 0 and 2 of T at
# several stream counts, then GPU tests + bench with each encoder variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R/tools
: > $O/gtab.log
for k in 0 2; do
  for n in 1024 4096 16384; do
    for b in enc_micro_np enc_micro_g enc_micro_g32; do
      echo "== $b plane $k n $n" >> $O/gtab.log
      timeout -k 10 60 ./$b fixtures/f32_p$k.bin fixtures/f32_p$k.out 5 $n >> $O/gtab.log 2>&1 || { echo "micro failed"; cat $O/gtab.log; exit 1; }
    done
  done
done
cd $R
for mode in 0 1; do
  export B2H_ENC_GTAB=$mode
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_gtab$mode.log 2>&1 || { echo "tests failed (gtab=$mode)"; tail -40 $O/gpu_tests_gtab$mode.log; exit 1; }
  tail -1 $O/gpu_tests_gtab$mode.log
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_gtab$mode.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_gtab$mode.log; exit 1; }
  tail -1 $O/bench_gtab$mode.log
done
