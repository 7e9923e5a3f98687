#!/bin/bash
# round 5: NP=8 rehearsal (gloo, one card, 1M rows per rank) under rocprofv3 kernel + memory-copy traces:
# the step's merges (shard_merge_kernel, no sort kernels) and its host<->device copies
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/np8t; export TMPDIR=/tmp
CM_DIST_BACKEND=gloo CM_BENCH_DEVICE=0 timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/np8t/tr -o np8 --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 8 --docs-per-gpu 1000000 --steps 5 --warmup 2 --e5-other-leg 0 --dense-legs 0 --cpu-baseline 0 --ingest-leg 0 > gpurun_out/np8t/np8.log 2>&1 || { tail -30 gpurun_out/np8t/np8.log; exit 1; }
grep "steps in" gpurun_out/np8t/np8.log | head -2 | cut -c1-200
ls gpurun_out/np8t/tr | head
