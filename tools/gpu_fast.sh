# Fast-mode check: its tests, then the T bench in both encoder modes (no CPU leg).
TAG=${1:-fast}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fast_mode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fast_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/fast_tests_$TAG.log; exit 1; }
tail -2 $O/fast_tests_$TAG.log
timeout -k 10 300 python -u bench.py --lz-mode fast --no-cpu-baseline > $O/bench_fast_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_fast_$TAG.log; exit 1; }
tail -1 $O/bench_fast_$TAG.log
echo DONE
