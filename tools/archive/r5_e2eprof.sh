#!/bin/bash
# round 5: host profile of the drop-in retrieve_batch at 1M chunks (cProfile over the timed calls)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2ep; export TMPDIR=/tmp
CM_E2E_PROFILE=1 timeout -k 10 600 python -u bench.py --mode e2e --docs-per-gpu 1000000 --e2e-construct 0 --steps 20 --out gpurun_out/e2ep/e2e.json > gpurun_out/e2ep/e2e.log 2>&1 || { tail -40 gpurun_out/e2ep/e2e.log; exit 1; }
grep -E "q/s|retrieve\(\)" gpurun_out/e2ep/e2e.log | cut -c1-200
