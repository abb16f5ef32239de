bash tools/gpu_job.sh r5f tests rp_c4 && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 python3 -u tools/bench_configs.py --only C4 --lz-mode fast --steps 5 > gpurun_out/r5f_c4_fast.log 2>&1 && \
timeout -k 10 300 python3 -u tools/bench_configs.py --only C4 --lz-mode exact --steps 5 > gpurun_out/r5f_c4_exact.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5f_bench.log 2>&1 && \
tail -1 gpurun_out/r5f_c4_fast.log && tail -1 gpurun_out/r5f_c4_exact.log && tail -1 gpurun_out/r5f_bench.log | cut -c1-400
