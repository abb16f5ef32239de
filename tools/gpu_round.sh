# Round measurement on the GPU box: GPU parity tests, the full bench (both BloscLZ modes, CPU
# baseline), a rocprofv3 kernel-trace/stats run of the bench in each mode, and HBM-traffic PMC
# passes over the fast-mode bench (FETCH_SIZE and WRITE_SIZE each in a pass of their own).  Every
# GPU step has its own limit and the chain stops at the first failure.
#   bash tools/gpu_round.sh <tag> [skip-tests]
TAG=${1:-r2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  echo "tests..."
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_$TAG.log; exit 1; }
  tail -3 $O/gpu_tests_$TAG.log
fi
echo "bench..."
timeout -k 10 500 python -u bench.py > $O/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_$TAG.log; exit 1; }
tail -1 $O/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
for mode in fast exact; do
  echo "rocprof stats $mode..."
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_${TAG}_$mode -o run -- python3 -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --lz-mode $mode > $O/rp_${TAG}_$mode.log 2>&1 || { echo "rocprof failed"; tail -30 $O/rp_${TAG}_$mode.log; exit 1; }
  tail -1 $O/rp_${TAG}_$mode.log | cut -c1-300
done
# HBM traffic per launch, fast mode (tag TAG) and exact mode (tag TAGx)
for mode in fast exact; do
  T=$TAG; [ $mode = exact ] && T=${TAG}x
  for ctr in FETCH_SIZE WRITE_SIZE; do
    echo "pmc $mode $ctr..."
    timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-include-regex "k_encode|k_decode|k_ffilter|k_dfilter|k_scatter" --output-format csv \
        -d $O/pmc_${T}_$ctr -o run -- python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --lz-mode $mode > $O/pmc_${T}_$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -20 $O/pmc_${T}_$ctr.log; exit 1; }
  done
  python3 $R/tools/pmc_traffic.py $O $T $O/pmc_traffic_$T.json $mode > /dev/null && echo "traffic summary: gpurun_out/pmc_traffic_$T.json"
done
echo DONE
