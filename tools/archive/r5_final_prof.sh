#!/bin/bash
# round 5 final tree: PMC traffic of K1q B=256 and K2a B=256, NP=8 rehearsal (gloo, one card), NP=2 kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/fprof gpurun_out/mgpu; export TMPDIR=/tmp
ROUND=r05c ONLY="dense_q8_B256 bm25_B256" bash tools/pmc_traffic.sh || exit 1
cat gpurun_out/pmc_traffic_r05c.txt
NP=8 DOCS=1000000 CPUB=1 TMO=600 bash tools/mgpu_rehearsal.sh || exit 1
CM_DIST_BACKEND=gloo CM_BENCH_DEVICE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fprof/np2 -o np2 --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --docs-per-gpu 1000000 --steps 5 --warmup 2 --e5-other-leg 0 --dense-legs 0 --cpu-baseline 0 --ingest-leg 0 > gpurun_out/fprof/np2.log 2>&1 || { tail -30 gpurun_out/fprof/np2.log; exit 1; }
python3 tools/kstats.py gpurun_out/fprof/np2 > gpurun_out/fprof/np2_kernels.txt && grep -ciE "sort|radix" gpurun_out/fprof/np2_kernels.txt; grep -E "shard_merge|tseed|merge_small" gpurun_out/fprof/np2_kernels.txt | cut -c1-150
