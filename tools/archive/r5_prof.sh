#!/bin/bash
# round 5 evidence: NP=8 rehearsal (gloo, one card), NP=2 rehearsal under a kernel trace (the merge kernel,
# no torch sorts), headline-only kernel trace (deferred fallback / re-rank times), PMC traffic of K1q-s B=16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/prof gpurun_out/mgpu; export TMPDIR=/tmp
NP=8 DOCS=1000000 CPUB=1 TMO=600 bash tools/mgpu_rehearsal.sh || exit 1
CM_DIST_BACKEND=gloo CM_BENCH_DEVICE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/np2 -o np2 --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --docs-per-gpu 1000000 --steps 5 --warmup 2 --e5-other-leg 0 --dense-legs 0 --cpu-baseline 0 --ingest-leg 0 > gpurun_out/prof/np2.log 2>&1 || { tail -30 gpurun_out/prof/np2.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof/np2 > gpurun_out/prof/np2_kernels.txt && head -40 gpurun_out/prof/np2_kernels.txt | cut -c1-150
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/hl -o hl --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/prof/bench_hl.json > gpurun_out/prof/bench_hl.log 2>&1 || { tail -30 gpurun_out/prof/bench_hl.log; exit 1; }
python3 tools/kstats.py gpurun_out/prof/hl > gpurun_out/prof/hl_kernels.txt && head -30 gpurun_out/prof/hl_kernels.txt | cut -c1-150
ROUND=r05 ONLY="dense_q8s_B16" bash tools/pmc_traffic.sh || exit 1
cat gpurun_out/pmc_traffic_r05.txt
