# exact-mode encoder shapes (B2H_ENC_MODE): LDS-table / global-table waves per workgroup
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in glb hyb3; do
  B2H_ENC_MODE=$m timeout -k 5 200 python -u bench.py --lz-mode exact --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4q_$m.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/r4q_$m.log; exit 1; }
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r4q_$m.log') if l.startswith('{')][0]; print('$m', d['modes'])"
done
