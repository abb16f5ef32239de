# A/B on one box: the previous library (lib_ab) vs the current one, T bench (fast) and C4 fast, alternating
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 1 2; do
  for v in prev cur; do
    if [ $v = prev ]; then export B2H_LIB=$GRAFT_REPO_ROOT/c-blosc2_amd/lib_ab/libblosc2.so; else unset B2H_LIB; fi
    timeout -k 5 200 python -u bench.py --lz-mode fast --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r4ac_${v}_$k.log 2>&1 || { echo "$v failed"; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r4ac_${v}_$k.log') if l.startswith('{')][0]; print('$v', $k, d['value'], d['modes']['fast']['encode_ms'], d['modes']['fast']['decode_ms'])"
  done
done
for v in prev cur; do
  if [ $v = prev ]; then export B2H_LIB=$GRAFT_REPO_ROOT/c-blosc2_amd/lib_ab/libblosc2.so; else unset B2H_LIB; fi
  timeout -k 5 300 python -u tools/bench_configs.py --only C4 --lz-mode fast > gpurun_out/r4ac_c4_$v.log 2>&1 || { echo "c4 $v failed"; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r4ac_c4_$v.log') if l.startswith('{')][0]; print('c4 $v', d['compress_ms'], d['decompress_ms'], d['GiBps_c_plus_d'])"
done
