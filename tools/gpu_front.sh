# Encoder pull schedule sweep (B2H_ENC_FRONT): GPU tests in the default, then the T bench per value.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_front.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_front.log; exit 1; }
tail -1 $O/gpu_tests_front.log
for f in ${FRONTS:-0 2 3 4}; do
  B2H_ENC_FRONT=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_front_$f.log 2>&1 || { echo "bench failed ($f)"; tail -30 $O/bench_front_$f.log; exit 1; }
  echo "front $f: $(tail -1 $O/bench_front_$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "GiB/s encode", d["roofline"]["encode_ms"], "ms decode", d["roofline"]["decode_ms"])')"
done
