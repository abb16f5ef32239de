# A/B of fused-encode modes: smoke (fused == separate), the fused-launch tests, then tools/fuse_prof.py.
O=gpurun_out
mkdir -p $O
timeout -k 10 120 python -u tools/fuse_smoke.py > $O/ab_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/ab_smoke.log; exit 1; }
grep -v amdgpu.ids $O/ab_smoke.log
timeout -k 10 200 python -u -m pytest tests/test_fast_mode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/ab_tests.log; exit 1; }
tail -1 $O/ab_tests.log
timeout -k 10 200 python -u tools/fuse_prof.py ${@:-19 3} > $O/ab_prof.log 2>&1 || { echo "prof failed"; tail -20 $O/ab_prof.log; exit 1; }
grep -v amdgpu.ids $O/ab_prof.log
