# C4 block-0 scan variant: tests touching DELTA, then the C4 kernel profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "delta or ds or C4 or configs or schunk or parity" > gpurun_out/r4z_tests.log 2>&1 || { echo tests failed; tail -20 gpurun_out/r4z_tests.log; exit 1; }
tail -1 gpurun_out/r4z_tests.log
sed -i 's/rp_r4y_c4/rp_r4z_c4/g' tools/gpu_r4x.sh
bash tools/gpu_r4x.sh
