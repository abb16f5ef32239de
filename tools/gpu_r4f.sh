# round 4: frames, fast bench, then the whole GPU tier; stop at the first failure
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4f_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4f_$name.log)"; return $rc; }
step frames 200 python -u -m pytest tests/test_gpu_frame_schunk.py -x -q --timeout 120 --timeout-method thread || exit 1
step bench 240 python -u bench.py --steps 10 --warmup 3 --lz-mode both --no-cpu-baseline || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/r4f_bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'], d['config'].get('cratio'))"
step gputier 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
