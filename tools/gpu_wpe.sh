# Global-table encoder micro-benchmark at several occupancy targets (waves per SIMD).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R/tools
: > $O/wpe.log
for k in 0 2; do
  for b in enc_micro_g enc_micro_g_w5 enc_micro_g_w6 enc_micro_g_w8; do
    echo "== $b plane $k n 16384" >> $O/wpe.log
    timeout -k 10 60 ./$b fixtures/f32_p$k.bin fixtures/f32_p$k.out 5 16384 >> $O/wpe.log 2>&1 || { echo "micro failed"; cat $O/wpe.log; exit 1; }
  done
done
grep -A1 "==" $O/wpe.log | grep -v "^--" | paste - -
