#!/bin/bash
# round-3 final check on the GPU box: what the driver runs (pytest -m gpu, smoke, bench) + rocprofv3
# summary of the bench, then PMC traffic of K1c (B=256), K1s (B=16) and K2a (B=256) for the final binary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/round_check.sh || exit 1
ROUND=r03final bash tools/pmc_traffic.sh > gpurun_out/pmc_final.log 2>&1 || { tail -20 gpurun_out/pmc_final.log; exit 1; }
cat gpurun_out/pmc_traffic_r03final.txt
