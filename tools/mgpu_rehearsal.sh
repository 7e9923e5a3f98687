#!/bin/bash
# GPU (1 card): bench.py's N>1 path with NP ranks (default 2; 8 = BASELINE configs[4]'s split) on the
# same GPU over gloo (RCCL refuses two ranks per device) -> gpurun_out/mgpu/rehearsal_np$NP.log.
# Shard merges, row offsets, global BM25 stats, the pool all-to-all, recall@10 vs the oracle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/mgpu; export TMPDIR=/tmp
NP=${NP:-2}
LOG=gpurun_out/mgpu/rehearsal_np$NP.log
CM_DIST_BACKEND=gloo CM_BENCH_DEVICE=0 timeout -k 10 ${TMO:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $NP --docs-per-gpu ${DOCS:-2000000} --steps 5 --warmup 2 \
  --e5-other-leg 0 --dense-legs 0 --cpu-baseline ${CPUB:-1} --cpu-queries 16 \
  --out gpurun_out/mgpu/rehearsal_np$NP.json > $LOG 2>&1 || { tail -40 $LOG; exit 1; }
grep "\[bench\]" $LOG | tail -4 | cut -c1-200
tail -1 $LOG | cut -c1-300
