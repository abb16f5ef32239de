# GPU parity tests, the config benchmarks (C2/C3/C4/E2E) and the T bench, each under its own limit.
# Usage on the GPU box: bash tools/gpu_check.sh <tag> [configs]
TAG=${1:-chk}
CFG=${2:-C2,C3,C4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_$TAG.log; exit 1; }
tail -1 $O/gpu_tests_$TAG.log
timeout -k 10 500 python -u tools/bench_configs.py --only $CFG > $O/configs_$TAG.log 2>&1 || { echo "configs failed"; tail -30 $O/configs_$TAG.log; exit 1; }
grep '^{' $O/configs_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_$TAG.log; exit 1; }
tail -1 $O/bench_$TAG.log
