#!/bin/bash
# round 5: drop-in e2e at 10M (retrieve_batch q/s, single retrieve() p50, the construct-then-retrieve
# leg of ask_question with its cold open)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2e; export TMPDIR=${TMPDIR:-/tmp}
df -h "$TMPDIR" . | sed 's/^/[df] /'
free -g | sed 's/^/[mem] /'
N=${1:-10000000}
timeout -k 10 1100 python -u bench.py --mode e2e --docs-per-gpu $N --out gpurun_out/e2e/e2e_$N.json > gpurun_out/e2e/e2e_$N.log 2>&1 || { tail -40 gpurun_out/e2e/e2e_$N.log; exit 1; }
grep -E "retrieve|construct|cold open|saved|q/s" gpurun_out/e2e/e2e_$N.log | cut -c1-300
