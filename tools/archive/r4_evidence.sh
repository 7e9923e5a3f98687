#!/bin/bash
# GPU: round-4 evidence on the current tree: default bench (all legs, CPU baseline), headline-only
# kernel trace, K1q PMC traffic (FETCH / WRITE passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ev; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --out gpurun_out/ev/bench_default.json > gpurun_out/ev/bench_default.log 2>&1 || { tail -30 gpurun_out/ev/bench_default.log; exit 1; }
tail -1 gpurun_out/ev/bench_default.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/trace -o hl --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/ev/bench_hl.json > gpurun_out/ev/bench_hl.log 2>&1 || { tail -30 gpurun_out/ev/bench_hl.log; exit 1; }
grep "steps in" gpurun_out/ev/bench_hl.log | cut -c1-300
ROUND=r04b ONLY="dense_q8_B256" bash tools/pmc_traffic.sh || exit 1
cat gpurun_out/pmc_traffic_r04b.txt
