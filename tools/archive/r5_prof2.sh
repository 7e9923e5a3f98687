#!/bin/bash
# round 5 evidence on the final tree: headline kernel trace + step timeline, PMC traffic of K1q B=256 and
# K2a B=256, then the NP=8 rehearsal (gloo, one card, 1M rows per rank)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/prof2 gpurun_out/mgpu; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/hl -o hl --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/prof2/bench_hl.json > gpurun_out/prof2/bench_hl.log 2>&1 || { tail -30 gpurun_out/prof2/bench_hl.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof2/hl > gpurun_out/prof2/hl_kernels.txt && head -24 gpurun_out/prof2/hl_kernels.txt | cut -c1-150
grep "steps in" gpurun_out/prof2/bench_hl.log | cut -c1-200
ROUND=r05b ONLY="dense_q8_B256 bm25_B256" bash tools/pmc_traffic.sh || exit 1
cat gpurun_out/pmc_traffic_r05b.txt
NP=8 DOCS=1000000 CPUB=1 TMO=600 bash tools/mgpu_rehearsal.sh || exit 1
