# decoder ring size sweep (B2H_DEC_RING = log2 bytes) on T, both modes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 13 12 14; do
  B2H_DEC_RING=$r timeout -k 5 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4ae_$r.log 2>&1 || { echo "$r failed"; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r4ae_$r.log') if l.startswith('{')][0]; print('ring', $r, {m: (v['decode_ms'], v['value']) for m, v in d['modes'].items()})"
done
