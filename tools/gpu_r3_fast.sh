# round 3: fast-mode correctness + bench (fast only)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
timeout -k 10 200 python -u -m pytest tests/test_fast_mode.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode fast > gpurun_out/r3_${TAG}_bench.log 2>&1
rc=$?
tail -2 gpurun_out/r3_${TAG}_tests.log
python -c "
import json;d=json.loads(open('gpurun_out/r3_${TAG}_bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'])" || true
exit $rc
