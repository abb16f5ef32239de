# round 4 diagnostics + checks, one GPU call; every step bounded, stop at the first failure
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4b_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4b_$name.log)"; return $rc; }
B2H_LIB=c-blosc2_amd/lib_trace/libblosc2.so B2H_TRACE_WG=3 B2H_DIAG_KEEP=0:1 B2H_FUSE=0 step trace 60 python -u tools/diag_fuse.py 1 16 || exit 1
grep -E "^wg|^late" gpurun_out/r4b_trace.log | head -20
B2H_DIAG_KEEP=0:1 B2H_FUSE=0 step prod_blk 60 python -u tools/diag_fuse.py 1 16 || exit 1
B2H_FUSE=0 step prod24 90 python -u tools/diag_fuse.py 24 0 || exit 1
step frames 200 python -u -m pytest tests/test_gpu_frame_schunk.py -x -q --timeout 120 --timeout-method thread || exit 1
step fasttests 300 python -u -m pytest tests/test_fast_mode.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
