# round 4: the restructured fast encoder (uniform run branch, single-exit loops) on the inputs that
# hung, then the batches, the fast-mode tests, the frame tests and the fast bench; stop at the first failure
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1 t=$2; shift 2; timeout -k 5 $t "$@" > gpurun_out/r4e_$name.log 2>&1; local rc=$?; echo "$name rc $rc: $(tail -n 1 gpurun_out/r4e_$name.log)"; return $rc; }
B2H_FUSE=0 step plane3 30 python -u tools/diag_stream.py 16 0 3 || exit 1
B2H_FUSE=0 step planes 30 python -u tools/diag_stream.py 16 0 0,1,2,3 || exit 1
B2H_FUSE=0 step blk0 40 python -u tools/diag_fuse.py 1 16 || exit 1
for f in 0 3 83; do B2H_FUSE=$f step b24_$f 90 python -u tools/diag_fuse.py 24 0 || exit 1; done
step fasttests 300 python -u -m pytest tests/test_fast_mode.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step frames 200 python -u -m pytest tests/test_gpu_frame_schunk.py -x -q --timeout 120 --timeout-method thread || exit 1
step bench 200 python -u bench.py --steps 10 --warmup 3 --lz-mode fast --no-cpu-baseline || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/r4e_bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'], d['config'].get('cratio'))"
