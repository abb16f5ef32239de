# Same-box A/B of the fast matcher (diagnostic): T fast mode with the current library and with
# variants/libblosc2_oldm.so (the round-4 matcher: a 60-byte compare at every position), alternated.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
for r in 1 2; do
  for cfg in "new:" "old:B2H_LIB=variants/libblosc2_oldm.so"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --lz-mode fast > $O/r5ab_$name$r.log 2>&1
    echo "== $name $r"; tail -1 $O/r5ab_$name$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['modes']['fast'])"
  done
done
