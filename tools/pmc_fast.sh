# SQ instruction / wait counters of the fast-mode micro-benchmark (one rocprofv3 pass per group).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_fast1 -o run -- $R/tools/fast_micro $R/tools/fixtures/f32_p2.bin 5 13 > $O/pmc_fast1.log 2>&1 || { echo pass1 failed; tail $O/pmc_fast1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d $O/pmc_fast2 -o run -- $R/tools/fast_micro $R/tools/fixtures/f32_p2.bin 5 13 > $O/pmc_fast2.log 2>&1 || { echo pass2 failed; tail $O/pmc_fast2.log; exit 1; }
echo DONE
