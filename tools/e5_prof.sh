#!/bin/bash
# GPU: rocprofv3 kernel stats of the E5 query-encode probe -> gpurun_out/e5prof/summary.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e5prof; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e5prof/raw -o e5 --output-format csv -- python3 tools/e5_probe.py > gpurun_out/e5prof/log.txt 2>&1 || { tail -20 gpurun_out/e5prof/log.txt; exit 1; }
f=$(find gpurun_out/e5prof/raw -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY' > gpurun_out/e5prof/summary.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:25]:
    print(f"{r['Name'][:90]:90s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:8.1f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
PY
cat gpurun_out/e5prof/summary.txt
