# Round measurement on the GPU box: GPU parity tests, the full bench (with CPU baseline), a
# rocprofv3 kernel-trace/stats run of the same bench, and HBM-traffic PMC passes over the T bench
# (FETCH_SIZE and WRITE_SIZE each in a pass of their own).  Every GPU step has its own limit and
# the chain stops at the first failure.   Usage: bash tools/gpu_round.sh <tag>
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "tests..."
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_$TAG.log; exit 1; }
tail -3 $O/gpu_tests_$TAG.log
echo "bench..."
timeout -k 10 400 python -u bench.py > $O/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_$TAG.log; exit 1; }
tail -1 $O/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
echo "rocprof stats..."
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_$TAG -o run -- python3 -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/rp_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $O/rp_$TAG.log; exit 1; }
tail -1 $O/rp_$TAG.log
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "pmc $ctr..."
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-include-regex "k_encode|k_decode|k_ffilter|k_dfilter|k_scatter" --output-format csv \
      -d $O/pmc_${TAG}_$ctr -o run -- python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_${TAG}_$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -20 $O/pmc_${TAG}_$ctr.log; exit 1; }
done
python3 $R/tools/pmc_traffic.py $O $TAG $O/pmc_traffic_$TAG.json > /dev/null && echo "traffic summary: gpurun_out/pmc_traffic_$TAG.json"
echo DONE
