# round 4: decoder frontier rounds -- GPU tier, then bench in both modes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4r_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4r_$name.log | cut -c1-300)"; return $rc; }
step gputier 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step bench 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit 1
