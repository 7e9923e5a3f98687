#!/bin/bash
# GPU: E5 query encode alone (bench shape, bf16): variant timings + per-kernel rocprof stats.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/e5_probe.py 2>&1 | grep ms
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e5prof -o run --output-format csv -- python3 tools/e5_probe.py > gpurun_out/e5prof.log 2>&1 || { tail -5 gpurun_out/e5prof.log; exit 1; }
f=$(find gpurun_out/e5prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{float(r["AverageNs"])/1e3:8.1f} us x {r["Calls"]:>5}  {r["Name"][:100]}')
PY
