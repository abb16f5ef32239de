# Encoder diagnostics on the GPU box: per-plane micro-benchmark (tools/enc_micro, built on the
# CPU side) on the four T planes, then per-plane window/cycle statistics of the batch encoder.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R/tools
for k in 0 1 2 3; do
  echo "== plane $k" >> $O/encdiag.log
  timeout -k 10 60 ./enc_micro fixtures/f32_p$k.bin fixtures/f32_p$k.out 5 >> $O/encdiag.log 2>&1 || { echo "enc_micro failed"; tail $O/encdiag.log; exit 1; }
done
cd $R
timeout -k 10 120 python -u tests/prof_encode.py 64 >> $O/encdiag.log 2>&1 || { echo "prof_encode failed"; exit 1; }
cat $O/encdiag.log
