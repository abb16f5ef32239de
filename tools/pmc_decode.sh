# PMC passes over k_decode (see pmc_encode.sh).  Usage: bash tools/pmc_decode.sh [nchunks]
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-64}
mkdir -p $R/gpurun_out/pmcd
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_IFETCH"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-include-regex "k_decode" --output-format csv \
      -d $R/gpurun_out/pmcd/p$i -o run -- python3 $R/tests/prof_decode.py $N > $R/gpurun_out/pmcd/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $set"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit $rc ;; esac
done
echo PMC_DONE
