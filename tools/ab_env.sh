# Same-box A/B of environment settings (diagnostic): T bench in one mode, the default environment
# against each "NAME=VALUE[,NAME=VALUE]" setting given, alternated twice.
#   bash tools/ab_env.sh <tag> <fast|exact> <setting> [<setting> ...]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
TAG=$1; MODE=$2; shift 2
for r in 1 2; do
  k=0
  for set in cur "$@"; do
    envs=""; [ "$set" != cur ] && envs="${set//,/ }"
    env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --lz-mode $MODE > $O/${TAG}_$k$r.log 2>&1
    echo "== $set $r"; tail -1 $O/${TAG}_$k$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['modes']['$MODE']; print(d['value'], m['encode_ms'], m['decode_ms'], m['compress_ms'])"
    k=$((k + 1))
  done
done
