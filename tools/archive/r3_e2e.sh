#!/bin/bash
# drop-in retrieve_batch end to end at the configured corpus size (device-resident batch path),
# then the N=2 rehearsal (recall diagnostics)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2e; export TMPDIR=/tmp
timeout -k 10 ${E2E_LIMIT:-900} python -u bench.py --mode e2e --docs-per-gpu ${DOCS:-10000000} --steps 10 --warmup 2 --out gpurun_out/e2e/e2e.json > gpurun_out/e2e/e2e.log 2>&1 || { tail -30 gpurun_out/e2e/e2e.log; exit 1; }
grep "\[bench\]" gpurun_out/e2e/e2e.log | cut -c1-300
if [ "${MGPU:-1}" = 1 ]; then DOCS=1000000 bash tools/mgpu_rehearsal.sh > gpurun_out/e2e/mgpu.txt 2>&1 || { tail -20 gpurun_out/e2e/mgpu.txt; exit 1; }; grep -E "recall|mismatch|gpu lists" gpurun_out/mgpu/rehearsal.log | cut -c1-1500; fi
