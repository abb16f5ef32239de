# C4 kernel profile (exact mode): where the decompress time goes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rp_r4y_c4 -o run -- python3 -u $GRAFT_REPO_ROOT/tools/bench_configs.py --only C4 --lz-mode exact --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/rp_r4y_c4.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/rp_r4y_c4.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/rp_r4y_c4.log | cut -c1-300
