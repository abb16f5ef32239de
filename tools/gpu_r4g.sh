# round 4: the round-3 tile encoder with the uniform-branch fixes: batches, the whole GPU tier, the default bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4g_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4g_$name.log)"; return $rc; }
for f in 0 83; do B2H_FUSE=$f step b24_$f 90 python -u tools/diag_fuse.py 24 0 || exit 1; done
step gputier 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step bench 300 python -u bench.py || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/r4g_bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'], d['config'].get('cratio'), d.get('cpu_baseline'))"
