#!/bin/bash
# Round 6: the drop-in API at 10M chunks (retrieve_batch, retrieve() latency by filter, construct-then-retrieve
# with the tail diagnostics, cold open), then C3's end-to-end ingest at 1M chunks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${E2E:-1}" = "1" ]; then
  timeout -k 10 900 python -u bench.py --mode e2e --docs-per-gpu 10000000 --steps 10 --warmup 2 --out gpurun_out/e2e_10m.json > gpurun_out/e2e_10m.log 2>&1 || { echo "e2e failed"; tail -30 gpurun_out/e2e_10m.log; exit 1; }
  grep "\[bench\]" gpurun_out/e2e_10m.log | tail -14
fi
if [ "${INGEST:-1}" = "1" ]; then
  timeout -k 10 1000 python -u bench.py --docs-per-gpu 1000000 --steps 5 --warmup 2 --dense-legs 0 --e5-other-leg 0 --cpu-baseline 0 --varlen-chunks 16384 --ingest-e2e-chunks 1048576 --ingest-e2e-file-chunks 65536 --out gpurun_out/ingest_1m.json > gpurun_out/ingest_1m.log 2>&1 || { echo "ingest failed"; tail -30 gpurun_out/ingest_1m.log; exit 1; }
  grep "\[bench\]" gpurun_out/ingest_1m.log | tail -12
fi
