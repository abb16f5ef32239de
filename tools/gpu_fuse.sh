# Fused fast-mode encode check: its tests first, then the GPU suite, then the bench with and
# without the fused launch (B2H_FUSE=0).  Every GPU step has its own limit; stops at the first failure.
# Usage: bash tools/gpu_fuse.sh <tag>
TAG=${1:-fuse}
O=gpurun_out
mkdir -p $O
echo "smoke..."
B2H_FUSE_TRACE=1 timeout -k 10 120 python -u tools/fuse_smoke.py > $O/fuse_smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -30 $O/fuse_smoke_$TAG.log; exit 1; }
cat $O/fuse_smoke_$TAG.log | grep -v amdgpu.ids
echo "fast-mode tests..."
timeout -k 10 300 python -u -m pytest tests/test_fast_mode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fuse_tests_$TAG.log 2>&1 || { echo "fast tests failed"; tail -40 $O/fuse_tests_$TAG.log; exit 1; }
tail -2 $O/fuse_tests_$TAG.log
echo "bench fused..."
timeout -k 10 300 python -u bench.py --no-cpu-baseline --lz-mode both > $O/bench_fused_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_fused_$TAG.log; exit 1; }
tail -1 $O/bench_fused_$TAG.log
echo "bench separate..."
B2H_FUSE=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --lz-mode fast > $O/bench_sep_$TAG.log 2>&1 || { echo "bench sep failed"; tail -30 $O/bench_sep_$TAG.log; exit 1; }
tail -1 $O/bench_sep_$TAG.log
echo "all GPU tests..."
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_$TAG.log; exit 1; }
tail -3 $O/gpu_tests_$TAG.log
echo DONE
