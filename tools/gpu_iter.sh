# One development iteration on the GPU box: encoder micro-benchmark on the four T planes
# (summary lines), GPU parity tests, and the bench without the CPU baseline.  Each GPU step has its
# own limit; the chain stops at the first failure.   Usage: bash tools/gpu_iter.sh <tag> [skip-tests]
TAG=${1:-it}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R/tools
: > $O/micro_$TAG.log
for k in 0 1 2 3; do
  echo "== plane $k" >> $O/micro_$TAG.log
  timeout -k 10 60 ./enc_micro fixtures/f32_p$k.bin fixtures/f32_p$k.out 5 >> $O/micro_$TAG.log 2>&1 || { echo "enc_micro failed rc=$?"; tail -20 $O/micro_$TAG.log; exit 1; }
done
grep -E "^==|blocks  1024|cycles/stream" $O/micro_$TAG.log | grep -v " 0 cycles" | awk '/blocks  1024/{p=1} /^==/{p=0; print; next} p'
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_$TAG.log; exit 1; }
  tail -2 $O/gpu_tests_$TAG.log
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_$TAG.log; exit 1; }
tail -1 $O/bench_$TAG.log
