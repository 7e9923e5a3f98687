#!/bin/bash
# GPU: kernel trace of the dense probe (per-kernel durations of one search pipeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o dp --output-format csv -- python3 tools/dense_probe.py --path ${DPATH:-3} --reps 5 > gpurun_out/dprof.log 2>&1 || { tail -20 gpurun_out/dprof.log; exit 1; }
f=$(find gpurun_out/dprof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/dense_kernel_stats.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/dense_kernel_stats.csv')):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
