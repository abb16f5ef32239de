# round 4: in-launch (DELTA, SHUFFLE) decode by rows: tests, C4 timing, T bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4i_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4i_$name.log)"; return $rc; }
step ds 300 python -u -m pytest tests/test_gpu_ds_decode.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread || exit 1
step c4 240 python -u tools/bench_configs.py --only C4 --lz-mode exact || exit 1
B2H_FUSE_UNSHUFFLE=0 step c4_nofuse 240 python -u tools/bench_configs.py --only C4 --lz-mode exact || exit 1
step bench 240 python -u bench.py --steps 10 --warmup 3 --lz-mode fast --no-cpu-baseline || exit 1
