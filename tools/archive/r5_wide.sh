#!/bin/bash
# round 5: K1q wide re-rank -- q8 tests + the certificate tests, then the bench's dense legs with the
# duplicate-cluster leg, wide re-rank on (product) vs off (CM_K1Q_WIDE=0: the exact scan)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/wide; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_engine.py -k "q8 or certificate or Q8" > gpurun_out/wide/pytest.log 2>&1 || { tail -40 gpurun_out/wide/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/wide/pytest.log | tail -2
for v in on off; do
  env $([ $v = off ] && echo CM_K1Q_WIDE=0) timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 --e5-other-leg 0 --ingest-leg 0 --cpu-baseline 0 --out gpurun_out/wide/bench_$v.json > gpurun_out/wide/bench_$v.log 2>&1 || { tail -20 gpurun_out/wide/bench_$v.log; exit 1; }
  grep -E "steps in|c4_dense|c2p|c4_dup" gpurun_out/wide/bench_$v.log | sed "s/^/$v /" | cut -c1-250
done
