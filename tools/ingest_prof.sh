#!/bin/bash
# GPU: C3 ingest encode (B=256, S=256, bf16) per-kernel rocprof stats.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ingprof -o run --output-format csv -- python3 bench.py --mode ingest --batch 256 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/ingprof.log 2>&1 || { tail -5 gpurun_out/ingprof.log; exit 1; }
tail -1 gpurun_out/ingprof.log | cut -c1-200
f=$(find gpurun_out/ingprof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms  {float(r["AverageNs"])/1e3:8.1f} us x {r["Calls"]:>5}  {r["Name"][:90]}')
PY
