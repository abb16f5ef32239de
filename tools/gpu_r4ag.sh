# fused fast launch knobs re-swept on the current kernel: B2H_ENC_FRONT (pull schedule), B2H_SHUF_LEAD
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local tag=$1; shift; env "$@" timeout -k 5 200 python -u bench.py --lz-mode fast --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r4ag_$tag.log 2>&1 || { echo "$tag failed"; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r4ag_$tag.log') if l.startswith('{')][0]; print('$tag', d['value'], d['modes']['fast']['encode_ms'])"; }
run base B2H_ENC_FRONT=2
run front1 B2H_ENC_FRONT=1
run front3 B2H_ENC_FRONT=3
run front4 B2H_ENC_FRONT=4
run lead256 B2H_SHUF_LEAD=256
run lead1024 B2H_SHUF_LEAD=1024
run base2 B2H_ENC_FRONT=2
