# A/B of one env setting: bench exact with the in-tree lib and lib_ab under ENVSET
set -o pipefail
cd $GRAFT_REPO_ROOT
export $1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode exact > gpurun_out/abe_new.log 2>&1 && \
B2H_LIB=$PWD/c-blosc2_amd/lib_ab/libblosc2.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode exact > gpurun_out/abe_old.log 2>&1
rc=$?
for f in new old; do python -c "
import json;d=json.loads(open('gpurun_out/abe_$f.log').read().strip().splitlines()[-1]);print('$f',d['value'],d['modes'])" || true; done
exit $rc
