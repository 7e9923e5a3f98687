#!/bin/bash
# GPU (1 card): bench.py's N>1 path with 2 ranks on the same GPU over gloo (RCCL refuses two ranks
# per device) -> gpurun_out/mgpu/rehearsal.log.  Shard merges, row offsets, global BM25 stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/mgpu; export TMPDIR=/tmp
CM_DIST_BACKEND=gloo CM_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --docs-per-gpu ${DOCS:-2000000} --steps 5 --warmup 2 \
  --cpu-baseline ${CPUB:-1} --cpu-queries 16 > gpurun_out/mgpu/rehearsal.log 2>&1 || { tail -40 gpurun_out/mgpu/rehearsal.log; exit 1; }
grep "\[bench\]" gpurun_out/mgpu/rehearsal.log | tail -4 | cut -c1-200
tail -1 gpurun_out/mgpu/rehearsal.log | cut -c1-300
