mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rp_r1c -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/rp_r1c.log 2>&1) && \
bash tools/pmc_encode.sh 64 > gpurun_out/pmc_driver.log 2>&1
echo DONE rc=$?
