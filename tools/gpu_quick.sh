# GPU tests + bench (no cpu baseline) + decode/encode timing; each step under its own limit.
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
echo DONE rc=$?
