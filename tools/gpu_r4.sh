# round 4: fast-mode (FM2) correctness vs the model + reference decode, then the T bench (fast only)
#   bash tools/gpu_r4.sh <tag> [tests-filter]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
K=${2:-}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fast_mode.py -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/r4_${TAG}_fast_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_${TAG}_fast_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|Timeout" gpurun_out/r4_${TAG}_fast_tests.log | head -20; exit $rc; }
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode fast --no-cpu-baseline > gpurun_out/r4_${TAG}_bench.log 2>&1
rc=$?
python -c "
import json;d=json.loads(open('gpurun_out/r4_${TAG}_bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'], d['config']['cratio'])" || tail -5 gpurun_out/r4_${TAG}_bench.log
exit $rc
