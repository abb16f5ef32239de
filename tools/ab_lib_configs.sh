# Same-box A/B of a library build variant on configs (diagnostic): tools/bench_configs.py with the
# current library and with c-blosc2_amd/lib_prof/libblosc2_<name>.so, alternated twice.
#   bash tools/ab_lib_configs.sh <tag> <name> <mode> <configs>
set -e
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1; NAME=$2; MODE=$3; CFG=$4
for r in 1 2; do
  for v in cur $NAME; do
    envs=""; [ $v != cur ] && envs="B2H_LIB=c-blosc2_amd/lib_prof/libblosc2_$v.so"
    env $envs timeout -k 10 300 python3 -u tools/bench_configs.py --only $CFG --lz-mode $MODE > gpurun_out/${TAG}_$v$r.log 2>&1
    echo "== $v $r $MODE: $(grep -o '"config": "C[0-9T][^:,]*\|decompress_ms": [0-9.]*\|compress_ms": [0-9.]*\|gpu_decompress_MBps": [0-9.]*\|gpu_compress_MBps": [0-9.]*' gpurun_out/${TAG}_$v$r.log | tr '\n' ' ')"
  done
done
