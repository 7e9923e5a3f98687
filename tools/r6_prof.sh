#!/bin/bash
# Round 6: kernel trace of the default bench, PMC traffic of K1q / K2a / K2b on the benched binary, and the
# K2b variant A/B in the headline step.  Each GPU step has its own limit; the chain stops at a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/bench_prof.sh || exit 1
ONLY="dense_q8_B256 bm25_B256 bm25b_B256" ROUND=r06 bash tools/pmc_traffic.sh || exit 1
cat gpurun_out/pmc_traffic_r06.txt
if [ "${AB:-1}" = "1" ]; then bash tools/r6_ab.sh || exit 1; fi
