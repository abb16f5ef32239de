#!/bin/bash
# SQ counter pass over the fast-mode encoder (one rocprofv3 --pmc run per build variant).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
for w in 2 1; do
  export B2H_FAST_WAVES=$w
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_enc_w$w -o pmc -- python3 bench.py --lz-mode fast --no-cpu-baseline --chunks 256 --steps 1 --warmup 1 > gpurun_out/pmc_enc_w$w.log 2>&1 || exit $?
done
