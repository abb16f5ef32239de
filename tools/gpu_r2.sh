# Round-2 check on the GPU box: all GPU tests, the T bench (with CPU baseline) and the C5 bench at
# N=1.  Every GPU step has its own limit; the chain stops at the first failure.
# Usage: bash tools/gpu_r2.sh <tag> [pytest -k expr]
TAG=${1:-r2}
K=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "tests..."
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_$TAG.log; exit 1; }
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_$TAG.log; exit 1; }
fi
tail -3 $O/gpu_tests_$TAG.log
echo "bench T..."
timeout -k 10 400 python -u bench.py > $O/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_$TAG.log; exit 1; }
tail -1 $O/bench_$TAG.log
echo "bench C5..."
timeout -k 10 400 python -u bench.py --workload C5 --steps 3 > $O/bench_c5_$TAG.log 2>&1 || { echo "bench C5 failed"; tail -30 $O/bench_c5_$TAG.log; exit 1; }
tail -1 $O/bench_c5_$TAG.log
echo DONE
