#!/bin/bash
# GPU: bench under rocprofv3 kernel trace -> gpurun_out/bench_kernel_stats.csv (+ the bench JSON line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/benchprof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --out gpurun_out/bench_prof.json > gpurun_out/bench_prof.log 2>&1 || { tail -20 gpurun_out/bench_prof.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_prof.log | tail -3
f=$(find gpurun_out/benchprof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/bench_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/bench_kernel_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:40]:
    print(f"{r['Name'][:80]:80s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
PY
