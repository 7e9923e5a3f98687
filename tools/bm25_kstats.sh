#!/bin/bash
# GPU: per-kernel times of the pruned BM25 search at the bench shape (rocprofv3 kernel trace).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bm25k -o run --output-format csv -- python3 tools/bm25_probe.py --paths 2 --reps 10 > gpurun_out/bm25k.log 2>&1 || { tail -5 gpurun_out/bm25k.log; exit 1; }
f=$(find gpurun_out/bm25k -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "bm25" in r["Name"] and int(r["Calls"]) >= 10]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows:
    print(f'{float(r["AverageNs"])/1e3:8.1f} us x {r["Calls"]:>4}  {r["Name"][:90]}')
PY
