# round 4: the in-launch (DELTA, SHUFFLE) decode: its tests, the whole GPU tier, the config benchmarks
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4h_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4h_$name.log)"; return $rc; }
step ds 300 python -u -m pytest tests/test_gpu_ds_decode.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread || exit 1
step gputier 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step cfg_exact 240 python -u tools/bench_configs.py --only C1,C3,C4 --lz-mode exact || exit 1
step cfg_fast 240 python -u tools/bench_configs.py --only C1,C3,C4 --lz-mode fast || exit 1
