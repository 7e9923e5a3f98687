#!/bin/bash
# GPU: device retrieve_batch with BM25 on a side stream -- drop-in parity tests, then the 10M e2e bench with the
# in-process A/B of single-query retrieve() latency (BM25 on the main stream: --e2e-ab-same-stream 1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2es; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 240 --timeout-method thread > gpurun_out/e2es/pytest.log 2>&1 || { tail -30 gpurun_out/e2es/pytest.log; exit 1; }
tail -1 gpurun_out/e2es/pytest.log
timeout -k 10 820 python -u bench.py --mode e2e --docs-per-gpu 10000000 --steps 10 --warmup 2 --e2e-ab-same-stream 1 --out gpurun_out/e2es/e2e.json > gpurun_out/e2es/e2e.log 2>&1 || { tail -30 gpurun_out/e2es/e2e.log; exit 1; }
grep "\[bench\]" gpurun_out/e2es/e2e.log | tail -12
