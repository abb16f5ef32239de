# One parameterised launcher for the GPU-box measurements (replaces the per-round gpu_r*.sh
# scripts).  Every GPU step has its own time limit; the chain stops at the first failure.
#   bash tools/gpu_job.sh <tag> <job> [<job> ...]
# jobs:
#   tests            pytest -m gpu (whole tier)
#   tests:<expr>     pytest -m gpu -k <expr>
#   bench            bench.py (default run: both modes + CPU baseline)
#   rp_fast|rp_exact rocprofv3 --kernel-trace --stats of bench.py in that mode
#   pmc_fast|pmc_exact  FETCH_SIZE / WRITE_SIZE passes of bench.py, summarised by pmc_traffic.py
#   stall_fast|stall_exact  SQ stall / issue / LDS-conflict passes over tests/prof_encode.py (T)
#   stall_c4         the same counters over C4's fused fast encoder launch
#   rp_c4|rp_c3|rp_c1  rocprofv3 kernel stats of tools/bench_configs.py for that config (fast mode)
#   pmc_c4           FETCH_SIZE / WRITE_SIZE over C4 (fast mode)
#   rpc_<cN>_<mode>  rocprof kernel stats of config cN in that mode (e.g. rpc_c3_exact)
#   pmcc_<cN>_<mode> FETCH_SIZE / WRITE_SIZE over config cN in that mode, summarised (pmc_traffic.py)
#   configs          tools/bench_configs.py, both modes
#   smoke            __graft_entry__.smoke()
#   frame_e2e        tools/frame_e2e.py (T frame file: write, open + decode warm / cold; host fan-out)
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
SQA="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
SQB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
for job in "$@"; do
  cd $R
  L="$O/${TAG}_$(echo "$job" | tr -c "A-Za-z0-9_\n" "_").log"
  echo "== $job"
  case $job in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$L" 2>&1 || fail "$job" "$L"
      tail -2 "$L" ;;
    tests:*)
      timeout -k 10 400 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 120 --timeout-method thread -k "${job#tests:}" > "$L" 2>&1 || fail "$job" "$L"
      tail -3 "$L" ;;
    frame_e2e)
      timeout -k 10 500 python -u tools/frame_e2e.py > "$L" 2>&1 || fail "$job" "$L"
      cat "$L" | grep measure ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$L" 2>&1 || fail "$job" "$L"
      tail -1 $L ;;
    bench)
      timeout -k 10 500 python -u bench.py > "$L" 2>&1 || fail "$job" "$L"
      tail -1 $L | cut -c1-600 ;;
    rp_fast|rp_exact)
      m=${job#rp_}; cd /tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_rp_$m -o run -- python3 -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --lz-mode $m > "$L" 2>&1 || fail "$job" "$L"
      tail -1 $L | cut -c1-400 ;;
    pmc_fast|pmc_exact)
      m=${job#pmc_}; cd /tmp
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-include-regex "k_encode|k_decode|k_ffilter|k_dfilter|k_scatter" --output-format csv \
          -d $O/pmc_${TAG}_${m}_$ctr -o run -- python3 -u $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --lz-mode $m > "$L" 2>&1 || fail "$job $ctr" $L
      done
      python3 $R/tools/pmc_traffic.py $O ${TAG}_${m} $O/${TAG}_pmc_traffic_$m.json $m > /dev/null && echo "traffic: gpurun_out/${TAG}_pmc_traffic_$m.json" ;;
    stall_fast|stall_exact)
      m=1; [ $job = stall_exact ] && m=0
      cd /tmp
      P="python3 $R/tests/prof_encode.py 1024 $m"
      timeout -s KILL 150 rocprofv3 --pmc $SQA --kernel-include-regex "k_encode" --output-format csv -d $O/${TAG}_${job}_a -o run -- $P > "$L" 2>&1 || fail "$job a" $L
      timeout -s KILL 150 rocprofv3 --pmc $SQB --kernel-include-regex "k_encode" --output-format csv -d $O/${TAG}_${job}_b -o run -- $P >> "$L" 2>&1 || fail "$job b" $L
      echo "stall counters: gpurun_out/${TAG}_${job}_{a,b}" ;;
    stall_c4)   # SQ stall / issue / LDS counters of C4's fused fast encoder launch
      cd /tmp
      P="python3 -u $R/tools/bench_configs.py --only C4 --lz-mode fast --steps 1"
      timeout -s KILL 200 rocprofv3 --pmc $SQA --kernel-include-regex "k_encode" --output-format csv -d $O/${TAG}_${job}_a -o run -- $P > "$L" 2>&1 || fail "$job a" $L
      timeout -s KILL 200 rocprofv3 --pmc $SQB --kernel-include-regex "k_encode" --output-format csv -d $O/${TAG}_${job}_b -o run -- $P >> "$L" 2>&1 || fail "$job b" $L
      echo "stall counters: gpurun_out/${TAG}_${job}_{a,b}" ;;
    rp_c4|rp_c3|rp_c1)
      c=${job#rp_}; C=${c^^}; cd /tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_rp_$c -o run -- python3 -u $R/tools/bench_configs.py --only $C --lz-mode fast --steps 3 > "$L" 2>&1 || fail "$job" "$L"
      tail -2 "$L" | cut -c1-400 ;;
    pmc_c4)
      cd /tmp
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-include-regex "k_" --output-format csv \
          -d $O/${TAG}_pmc_c4_$ctr -o run -- python3 -u $R/tools/bench_configs.py --only C4 --lz-mode fast --steps 1 > "$L" 2>&1 || fail "$job $ctr" $L
      done
      echo "c4 pmc: gpurun_out/${TAG}_pmc_c4_*" ;;
    rpc_*)   # rpc_<c1..c4>_<fast|exact>: rocprof kernel stats of one config in one mode
      x=${job#rpc_}; c=${x%_*}; m=${x#*_}; C=${c^^}; cd /tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_rp_${c}_$m -o run -- python3 -u $R/tools/bench_configs.py --only $C --lz-mode $m --steps 3 > "$L" 2>&1 || fail "$job" "$L"
      tail -1 "$L" | cut -c1-400 ;;
    pmcc_*)  # pmcc_<c1..c4>_<fast|exact>: FETCH_SIZE / WRITE_SIZE passes of one config, summarised (rename the json to rN_vK[x]_cN_pmc_traffic.json when committing)
      x=${job#pmcc_}; c=${x%_*}; m=${x#*_}; C=${c^^}; cd /tmp
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-include-regex "k_" --output-format csv \
          -d $O/pmc_${TAG}_$c${m}_$ctr -o run -- python3 -u $R/tools/bench_configs.py --only $C --lz-mode $m --steps 1 > "$L" 2>&1 || fail "$job $ctr" $L
      done
      python3 $R/tools/pmc_traffic.py $O ${TAG}_$c$m $O/${TAG}_pmc_traffic_${c}_$m.json $m "$C (tools/bench_configs.py --only $C)" > /dev/null && echo "traffic: gpurun_out/${TAG}_pmc_traffic_${c}_$m.json" ;;
    configs)
      for m in fast exact; do
        timeout -k 10 500 python3 -u tools/bench_configs.py --lz-mode $m > $O/${TAG}_configs_$m.log 2>&1 || fail "configs $m" $O/${TAG}_configs_$m.log
        tail -8 $O/${TAG}_configs_$m.log | cut -c1-300
      done ;;
    *) echo "unknown job $job"; exit 2 ;;
  esac
done
echo DONE
