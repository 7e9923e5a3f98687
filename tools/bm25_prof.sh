#!/bin/bash
# GPU: kernel trace of the 10M BM25 probe (per-kernel durations of one search pipeline).
#   PATHS=2 bash tools/bm25_prof.sh -> gpurun_out/bm25_kernel_stats.csv + summary on stdout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o bp --output-format csv -- python3 tools/bm25_probe.py --paths ${PATHS:-2} --reps 5 > gpurun_out/bprof.log 2>&1 || { tail -20 gpurun_out/bprof.log; exit 1; }
grep "docs=" gpurun_out/bprof.log
f=$(find gpurun_out/bprof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/bm25_kernel_stats.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/bm25_kernel_stats.csv')):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
