# A/B of the decoder's pull order (B2H_DEC_ORDER: 0 LZ / raw-first by class, 1 stream order):
# T in both BloscLZ modes, then C1/C3/C4 (tools/bench_configs.py).
O=gpurun_out
for m in 0 1; do
  for lz in fast exact; do
    B2H_DEC_ORDER=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --lz-mode $lz --steps 5 > $O/bench_order${m}_$lz.log 2>&1 || { echo "bench $m failed"; tail -5 $O/bench_order${m}_$lz.log; exit 1; }
    echo "order $m $lz: $(tail -1 $O/bench_order${m}_$lz.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); m=list(d["modes"].values())[-1]; print(d["value"], m["compress_ms"], m["decompress_ms"], m["decode_ms"])')"
  done
  B2H_DEC_ORDER=$m timeout -k 10 300 python -u tools/bench_configs.py --only C1,C3,C4 > $O/configs_order$m.log 2>&1 || { echo "configs $m failed"; tail -5 $O/configs_order$m.log; exit 1; }
  grep -v amdgpu.ids $O/configs_order$m.log | cut -c1-300
done
