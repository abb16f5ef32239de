# Occupancy elasticity of the fused fast encoder (diagnostic): T fast mode at the default build and
# tablog, tablog 12 (LDS for 14 workgroups per CU), and a 5-waves-per-SIMD build (<= 96 VGPRs).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
for cfg in "base13:" "base12:B2H_FAST_TABLOG=12" "wpe5_12:B2H_FAST_TABLOG=12 B2H_LIB=variants/libblosc2_wpe5.so" "wpe5_13:B2H_LIB=variants/libblosc2_wpe5.so"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --lz-mode fast > $O/r5s_$name.log 2>&1
  echo "== $name"; tail -1 $O/r5s_$name.log | cut -c1-900
done
