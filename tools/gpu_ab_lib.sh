# A/B: bench with the in-tree library vs c-blosc2_amd/lib_ab (a build of another revision)
set -o pipefail
cd $GRAFT_REPO_ROOT
MODE=${1:-exact}
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode $MODE > gpurun_out/ab_new.log 2>&1 && \
B2H_LIB=$PWD/c-blosc2_amd/lib_ab/libblosc2.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lz-mode $MODE > gpurun_out/ab_old.log 2>&1
rc=$?
for f in new old; do python -c "
import json;d=json.loads(open('gpurun_out/ab_$f.log').read().strip().splitlines()[-1]);print('$f',d['value'],d['modes'])" || true; done
exit $rc
