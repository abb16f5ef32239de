# C1 per-call path: kernel trace of blosc1_compress / blosc1_decompress calls on host buffers
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rp_r4af_c1 -o run -- python3 -u $GRAFT_REPO_ROOT/tools/bench_configs.py --only C1 --lz-mode exact --steps 1 > $GRAFT_REPO_ROOT/gpurun_out/rp_r4af_c1.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/rp_r4af_c1.log; exit 1; }
grep gpu_per_call $GRAFT_REPO_ROOT/gpurun_out/rp_r4af_c1.log | cut -c1-100; echo done
