# Same-box A/B of library variants on one tools/bench_configs.py config (diagnostic), alternated.
#   bash tools/ab_configs.sh <tag> <config> <lz-mode> <name> [<name> ...]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
TAG=$1; CFG=$2; MODE=$3; shift 3
for r in 1 2; do
  for name in cur "$@"; do
    envs=""; [ $name != cur ] && envs="B2H_LIB=variants/libblosc2_$name.so"
    env $envs timeout -k 10 300 python -u tools/bench_configs.py --only $CFG --lz-mode $MODE > $O/${TAG}_$name$r.log 2>&1
    echo "== $name $r"; tail -1 $O/${TAG}_$name$r.log | cut -c1-400
  done
done
