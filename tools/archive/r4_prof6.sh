#!/bin/bash
# GPU: kernel trace of the headline step (no side legs), K1q v6
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/prof6; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6/trace -o hl --output-format csv -- python3 -u bench.py --steps 10 --warmup 3 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/prof6/bench.json > gpurun_out/prof6/bench.log 2>&1 || { tail -30 gpurun_out/prof6/bench.log; exit 1; }
grep "steps in" gpurun_out/prof6/bench.log | cut -c1-200
f=$(find gpurun_out/prof6/trace -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:40]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
