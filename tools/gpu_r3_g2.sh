set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fast_mode.py -x -v --timeout 120 --timeout-method thread -k "small_grid or two_streams" > gpurun_out/r3_g2_harden.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_g2_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py --only E2E --steps 3 > gpurun_out/r3_g2_e2e.log 2>&1
echo rc=$?
