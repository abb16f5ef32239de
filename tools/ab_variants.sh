# Same-box A/B of library variants (diagnostic): T bench in one mode with the current library and
# with each variants/libblosc2_<name>.so given, alternated twice.
#   bash tools/ab_variants.sh <tag> <fast|exact> <name> [<name> ...]
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
TAG=$1; MODE=$2; shift 2
for r in 1 2; do
  for name in cur "$@"; do
    envs=""; [ $name != cur ] && envs="B2H_LIB=variants/libblosc2_$name.so"
    env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --lz-mode $MODE > $O/${TAG}_$name$r.log 2>&1
    echo "== $name $r"; tail -1 $O/${TAG}_$name$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['modes']['$MODE']; print(d['value'], m['encode_ms'], m['decode_ms'])"
  done
done
