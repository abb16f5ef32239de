# rocprofv3 kernel trace of the C4 config (delta+shuffle+BloscLZ int64 schunk) alone.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_c4 -o run -- python3 -u $R/tools/bench_configs.py --only ${CFG:-C4} --steps 2 > $O/rp_c4.log 2>&1 || { echo "rocprof failed"; tail -30 $O/rp_c4.log; exit 1; }
grep '^{' $O/rp_c4.log
python3 -c "
import csv
for r in csv.DictReader(open('$O/rp_c4/run_kernel_stats.csv')):
  if 'b2h' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
