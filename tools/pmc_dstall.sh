# Stall / issue breakdown of the decoder on T (tests/prof_decode.py, 1024 x 4 MiB chunks); $1 = mode.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
M=${1:-1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tests/prof_decode.py 1024 $M"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $O/dstall_m${M}_a -o run -- $P > $O/dstall_m${M}_a.log 2>&1 || { echo passA failed; tail $O/dstall_m${M}_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES --output-format csv -d $O/dstall_m${M}_b -o run -- $P > $O/dstall_m${M}_b.log 2>&1 || { echo passB failed; tail $O/dstall_m${M}_b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/dstall_m${M}_c -o run -- $P > $O/dstall_m${M}_c.log 2>&1 || { echo passC failed; tail $O/dstall_m${M}_c.log; exit 1; }
echo DONE
