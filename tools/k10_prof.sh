# K10 probe under rocprofv3 kernel trace (per-kernel average durations)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10prof; export TMPDIR=/tmp
K10_E5=0 timeout -k 10 300 python -u tools/k10_probe.py > gpurun_out/k10prof/probe.log 2>&1 || { tail -20 gpurun_out/k10prof/probe.log; exit 1; }
cat gpurun_out/k10prof/probe.log
K10_E5=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k10prof/rp -o k10 --output-format csv -- python3 tools/k10_probe.py > gpurun_out/k10prof/rp.log 2>&1 || { tail -20 gpurun_out/k10prof/rp.log; exit 1; }
f=$(find gpurun_out/k10prof/rp -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/k10prof/kernel_stats.csv
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/k10prof/kernel_stats.csv')))
for r in rows[:14]: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
