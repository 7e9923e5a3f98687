#!/bin/bash
# GPU: K1q epilogue split (tests vs appends) + K1q PMC traffic at 10M x 768, B = 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/k1q_abl2.sh || exit 1
ROUND=r04q ONLY="dense_q8_B256" bash tools/pmc_traffic.sh || exit 1
cat gpurun_out/pmc_traffic_r04q.txt
