set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/pmc_stall.sh 1 && bash tools/pmc_stall.sh 0
echo rc=$?
