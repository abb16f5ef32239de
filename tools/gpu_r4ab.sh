# fused (DELTA, SHUFFLE) job in the encoder launch: tests, then C4 fast / exact
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4ab_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4ab_$name.log | cut -c1-300)"; return $rc; }
step fused 400 python -u -m pytest tests/test_fast_mode.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused" || exit 1
step gputier 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step c4_fast 300 python -u tools/bench_configs.py --only C4 --lz-mode fast || exit 1
step bench 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit 1
