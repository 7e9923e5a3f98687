#!/bin/bash
# GPU: step schedule A/B with K1q (BM25 beside E5 = default | BM25 after E5, beside the dense search |
# serial | BM25 stream at high priority), headline-only legs, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/sched; export TMPDIR=/tmp
for rep in 1 2; do
for v in "default:" "after:--bm25-after-e5" "serial:--serial" "prio:--bm25-priority -1"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 $flags --out gpurun_out/sched/$name.json > gpurun_out/sched/$name.log 2>&1 || { tail -20 gpurun_out/sched/$name.log; exit 1; }
  echo "$name $(grep 'steps in' gpurun_out/sched/$name.log | cut -c1-140)"
done; done
