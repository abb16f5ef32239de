# A/B of launch knobs on the T bench (fast mode): each line "ENV=value ..." of the arguments is
# one run.  Usage: bash tools/gpu_ab_env.sh "" "B2H_DEC_RING=12" ...
O=gpurun_out
n=0
for cfg in "$@"; do
  n=$((n+1))
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --lz-mode fast --steps 5 > $O/ab_env_$n.log 2>&1 || { echo "[$cfg] failed"; tail -5 $O/ab_env_$n.log; exit 1; }
  echo "[$cfg] $(tail -1 $O/ab_env_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); m=d["modes"]["fast"]; print(d["value"], m["compress_ms"], m["decompress_ms"], m["encode_ms"], m["decode_ms"])')"
done
