# Stall / issue breakdown of the encoder kernels on T (tests/prof_encode.py, 1024 x 4 MiB chunks).
# One rocprofv3 pass per counter group; $1 = BloscLZ mode (1 fast, 0 exact).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
M=${1:-1}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tests/prof_encode.py 1024 $M"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/stall_m${M}_a -o run -- $P > $O/stall_m${M}_a.log 2>&1 || { echo passA failed; tail $O/stall_m${M}_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --output-format csv -d $O/stall_m${M}_b -o run -- $P > $O/stall_m${M}_b.log 2>&1 || { echo passB failed; tail $O/stall_m${M}_b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_IFETCH --output-format csv -d $O/stall_m${M}_c -o run -- $P > $O/stall_m${M}_c.log 2>&1 || { echo passC failed; tail $O/stall_m${M}_c.log; exit 1; }
echo DONE
