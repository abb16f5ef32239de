# round 4 final measurements: GPU tier, config benchmarks (C1 incl. the per-call path, C3, C4) in both
# modes, then the round profile (bench, rocprof stats both modes, PMC traffic)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4j_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4j_$name.log | cut -c1-300)"; return $rc; }
step gputier 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step cfg_exact 240 python -u tools/bench_configs.py --only C1,C3,C4 --lz-mode exact || exit 1
step cfg_fast 240 python -u tools/bench_configs.py --only C1,C3,C4 --lz-mode fast || exit 1
bash tools/gpu_round.sh r4_v2 skip-tests
