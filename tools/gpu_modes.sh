# Encoder workgroup shapes (B2H_ENC_MODE): GPU tests in the default shape, then the T bench in each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_modes.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests_modes.log; exit 1; }
tail -1 $O/gpu_tests_modes.log
for mode in ${MODES:-lds glb hyb1 hyb2 hyb3}; do
  B2H_ENC_MODE=$mode timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_mode_$mode.log 2>&1 || { echo "bench failed ($mode)"; tail -30 $O/bench_mode_$mode.log; exit 1; }
  echo "$mode: $(tail -1 $O/bench_mode_$mode.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "GiB/s encode", d["roofline"]["encode_ms"], "ms decode", d["roofline"]["decode_ms"])')"
done
