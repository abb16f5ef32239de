# round 3: fast-mode correctness (model + reference decode), encoder micro-benchmark, T bench (fast only)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fast_mode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_${TAG}_fast_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3_${TAG}_fast_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r3_${TAG}_fast_tests.log | head -20; exit $rc; }
timeout -k 5 60 tools/fast_micro tools/fixtures/f32_p2.bin 5 13 > gpurun_out/r3_${TAG}_fm_p2.log 2>&1 && \
timeout -k 5 60 tools/fast_micro tools/fixtures/f32_p0.bin 5 13 > gpurun_out/r3_${TAG}_fm_p0.log 2>&1 && \
grep blocks gpurun_out/r3_${TAG}_fm_p2.log gpurun_out/r3_${TAG}_fm_p0.log && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode fast --no-cpu-baseline > gpurun_out/r3_${TAG}_bench.log 2>&1
rc=$?
python -c "
import json;d=json.loads(open('gpurun_out/r3_${TAG}_bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'], d['config']['cratio'])" || tail -5 gpurun_out/r3_${TAG}_bench.log
exit $rc
