# round 3: full GPU test tier + bench (both BloscLZ modes)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_${TAG}_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_${TAG}_bench.log 2>&1
rc=$?
tail -3 gpurun_out/r3_${TAG}_tests.log
python -c "
import json;d=json.loads(open('gpurun_out/r3_${TAG}_bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'])" || true
exit $rc
