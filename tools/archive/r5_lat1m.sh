#!/bin/bash
# round 5: single retrieve() latency at 1M chunks with the host profile of the timed calls
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/lat; export TMPDIR=/tmp
CM_E2E_PROFILE_LAT=1 timeout -k 10 600 python -u bench.py --mode e2e --docs-per-gpu 1000000 --out gpurun_out/lat/e2e_1m.json > gpurun_out/lat/e2e_1m.log 2>&1 || { tail -40 gpurun_out/lat/e2e_1m.log; exit 1; }
grep -E "retrieve|q/s" gpurun_out/lat/e2e_1m.log | cut -c1-300
