# Decoder ring-size sweep: GPU tests at the default ring, the LZ-heavy tests at ring 12, then the
# T bench per ring size (B2H_DEC_RING).   Usage: bash tools/gpu_ring.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_ring.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests_ring.log; exit 1; }
tail -1 $O/gpu_tests_ring.log
B2H_DEC_RING=12 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "far or corrupt or golden or random or batch" > $O/gpu_tests_ring12.log 2>&1 || { echo "ring12 tests failed"; tail -30 $O/gpu_tests_ring12.log; exit 1; }
tail -1 $O/gpu_tests_ring12.log
for r in ${RINGS:-13 12}; do
  B2H_DEC_RING=$r timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_ring$r.log 2>&1 || { echo "bench failed $r"; tail -20 $O/bench_ring$r.log; exit 1; }
  echo "ring $r: $(tail -1 $O/bench_ring$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "enc", d["roofline"]["encode_ms"], "dec", d["roofline"]["decode_ms"])')"
done
