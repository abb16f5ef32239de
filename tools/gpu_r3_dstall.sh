set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/pmc_dstall.sh 1 && bash tools/pmc_dstall.sh 0 && \
B2H_DECODE_DEBUG=1 timeout -k 10 120 python3 tests/prof_decode.py 1024 1 > gpurun_out/dprof_m1.log 2>&1 && \
B2H_DECODE_DEBUG=1 timeout -k 10 120 python3 tests/prof_decode.py 1024 0 > gpurun_out/dprof_m0.log 2>&1 && \
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u tools/bench_configs.py --only E2E --steps 3 > gpurun_out/r3_e2e_nosdma.log 2>&1
echo rc=$?
