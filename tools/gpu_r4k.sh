# round 4: BloscLZ mode 2 (deep candidates) -- kernel vs model, ratios, speed on T / C1 / C3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4k_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4k_$name.log | cut -c1-400)"; return $rc; }
step fastmode 400 python -u -m pytest tests/test_fast_mode.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step bench_deep 200 python -u bench.py --lz-mode deep --steps 5 --warmup 2 --no-cpu-baseline || exit 1
step cfg_deep 240 python -u tools/bench_configs.py --only C1,C3 --lz-mode deep || exit 1
