cd $GRAFT_REPO_ROOT
for v in base mu8; do
  if [ $v = mu8 ]; then export B2H_LIB=$GRAFT_REPO_ROOT/c-blosc2_amd/lib/libblosc2_mu8.so; else unset B2H_LIB; fi
  timeout -k 10 300 python -u tools/bench_configs.py --only C4 --lz-mode fast --steps 5 > gpurun_out/r5x_c4_$v.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --lz-mode fast > gpurun_out/r5x_t_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r5x_c4_$v.log | cut -c1-330)"; echo "$v T $(tail -1 gpurun_out/r5x_t_$v.log | cut -c1-120)"
done
