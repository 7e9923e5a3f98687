#!/bin/bash
# round 5: the large-batch 192 x 192 pick -- GEMM accuracy / QKV planes / E5 tests, ingest encode
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/tilechk; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/tilechk/pytest.log 2>&1 || { tail -40 gpurun_out/tilechk/pytest.log; exit 1; }
tail -1 gpurun_out/tilechk/pytest.log
grep -E "K10 (65536|30000)" gpurun_out/tilechk/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/tilechk/ingest.log 2>&1 || { tail -20 gpurun_out/tilechk/ingest.log; exit 1; }
  echo "ingest $(tail -1 gpurun_out/tilechk/ingest.log | cut -c1-170)"
done
