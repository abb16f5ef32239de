# exact compare width for u32-position streams (C3)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4w_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4w_$name.log | cut -c1-250)"; return $rc; }
step gputier 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step cfg_exact 300 python -u tools/bench_configs.py --only C3 --lz-mode exact || exit 1
step cfg_exact2 300 python -u tools/bench_configs.py --only C3 --lz-mode exact || exit 1
