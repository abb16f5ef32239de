set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_g1_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_g1_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_g1_bench.log 2>&1
echo rc=$?
