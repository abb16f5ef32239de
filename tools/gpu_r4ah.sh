# end-to-end (host -> device -> host, PCIe-inclusive) on the final tree, and LZ4 / C2 configs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 5 400 python -u tools/bench_configs.py --only E2E,C2,LZ4 --lz-mode fast > gpurun_out/r4ah_fast.log 2>&1 || { echo failed; tail -20 gpurun_out/r4ah_fast.log; exit 1; }
grep '^{' gpurun_out/r4ah_fast.log | cut -c1-400
