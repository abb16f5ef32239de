# SQ PMC passes over the encoder micro-benchmark (plane 2 of T, 1024 streams); one rocprofv3 run
# per counter set, never combined with tracing.   Usage on the GPU box: bash tools/pmc_micro.sh <tag>
TAG=${1:-m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcm_$TAG
mkdir -p $O
cd $R/tools
for k in 0 2; do
  timeout -k 10 60 ./enc_micro_np fixtures/f32_p$k.bin fixtures/f32_p$k.out 5 1024 >> $O/np.log 2>&1 || exit 1
  timeout -k 10 60 ./enc_micro_np fixtures/f32_p$k.bin fixtures/f32_p$k.out 5 4096 >> $O/np.log 2>&1 || exit 1
done
cat $O/np.log
cd /tmp
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- $R/tools/enc_micro_np $R/tools/fixtures/f32_p2.bin $R/tools/fixtures/f32_p2.out 5 1024 > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
