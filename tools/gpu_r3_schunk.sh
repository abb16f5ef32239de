set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_schunk_api.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_schunk_tests.log 2>&1
echo rc=$?
