# round 4 final: configs in both modes on the final tree
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4v_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4v_$name.log | cut -c1-200)"; return $rc; }
step cfg_exact 300 python -u tools/bench_configs.py --only C1,C3,C4 --lz-mode exact || exit 1
step cfg_fast 300 python -u tools/bench_configs.py --only C1,C3,C4 --lz-mode fast || exit 1
