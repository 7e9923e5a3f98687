#!/bin/bash
# round 5: drop-in retrieve_batch at 10M -- default vs full-LDS K1q vs 1024-thread BM25 merge vs both (env A/B in one process)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2eab; export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 1100 python -u bench.py --mode e2e --docs-per-gpu 10000000 --e2e-construct 0 --steps 20 \
  --e2e-ab-env "CM_K1Q_SHARED_LDS=0;CM_BM25_MERGE_SMALL=0;CM_K1Q_SHARED_LDS=0,CM_BM25_MERGE_SMALL=0" \
  --out gpurun_out/e2eab/e2e.json > gpurun_out/e2eab/e2e.log 2>&1 || { tail -40 gpurun_out/e2eab/e2e.log; exit 1; }
grep -E "A/B|retrieve|q/s" gpurun_out/e2eab/e2e.log | cut -c1-300
