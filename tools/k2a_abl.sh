#!/bin/bash
# GPU: K2a ablations at 10M (results are NOT valid under CM_BM25_DEBUG; timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/abl
for d in ${DBG:-0 16 32 48}; do
  CM_BM25_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abl/k2a_$d -o k --output-format csv -- python3 tools/bm25_probe.py --paths 2 --reps 3 > gpurun_out/abl/k2a_$d.log 2>&1 || { tail -5 gpurun_out/abl/k2a_$d.log; exit 1; }
  f=$(find gpurun_out/abl/k2a_$d -name '*kernel_stats.csv' | head -1)
  echo "dbg=$d $(python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'tail_kernel' in r['Name']: print('tail_us', round(float(r['AverageNs'])/1e3,1))
")"
done
