# rocprofv3 kernel stats of cfg5's rank-0 shard for N = 2 and 8 (tools/shard_prof.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/shard
for n in 1 2 8; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/shard/n$n -o kt --output-format csv -- python3 tools/shard_prof.py $n 20 > gpurun_out/shard/n$n.log 2>&1 || { echo "n$n failed"; tail -5 gpurun_out/shard/n$n.log; exit 1; }
  grep "{" gpurun_out/shard/n$n.log | tail -1
  f=$(find gpurun_out/shard/n$n -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
rows = list(csv.DictReader(open('$f')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:10]: print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
"
done
