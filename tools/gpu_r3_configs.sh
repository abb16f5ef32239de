# round 3: every BASELINE configuration in both BloscLZ modes (tools/bench_configs.py), C5 at N=1, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_configs.py --only C1,C2,C3,C4,E2E,LZ4 --lz-mode exact > gpurun_out/r3_cfg_exact.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_configs.py --only C1,C3,C4,E2E --lz-mode fast > gpurun_out/r3_cfg_fast.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload C5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3_c5.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1
rc=$?
grep -h '^{' gpurun_out/r3_cfg_exact.log gpurun_out/r3_cfg_fast.log | cut -c1-300
tail -1 gpurun_out/r3_c5.log | cut -c1-300
tail -2 gpurun_out/r3_smoke.log
exit $rc
