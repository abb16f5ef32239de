# round 3: exact-mode encoder change -- byte parity with the oracle / reference, micro-benchmark, T bench (exact)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_${TAG}_exact_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r3_${TAG}_exact_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r3_${TAG}_exact_tests.log | head -20; exit $rc; }
timeout -k 5 60 tools/enc_micro tools/fixtures/f32_p2.bin tools/fixtures/f32_p2.out > gpurun_out/r3_${TAG}_em.log 2>&1 && head -16 gpurun_out/r3_${TAG}_em.log && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode exact --no-cpu-baseline > gpurun_out/r3_${TAG}_bench_exact.log 2>&1
rc=$?
python -c "
import json;d=json.loads(open('gpurun_out/r3_${TAG}_bench_exact.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['modes'])" || tail -5 gpurun_out/r3_${TAG}_bench_exact.log
exit $rc
