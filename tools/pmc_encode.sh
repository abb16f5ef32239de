# PMC passes over k_encode (one rocprofv3 run per counter set; never combined with tracing).
# Usage on the GPU box: bash tools/pmc_encode.sh [nchunks]   -> gpurun_out/pmc/p<i>/...
# Stops at the first pass that faults / aborts / times out; a pass rejected for an unknown
# counter name (exit 1) is skipped.
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-64}
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum" \
           "SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-include-regex "k_encode" --output-format csv \
      -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/tests/prof_encode.py $N > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $set"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit $rc ;; esac
done
echo PMC_DONE
