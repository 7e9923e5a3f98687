#!/bin/bash
# GPU: step composition — default (overlapped), serial BM25, no E5, dense only.  -> gpurun_out/compose/*.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/compose; export TMPDIR=/tmp
for v in ${VARIANTS:-default: serial:--serial noe5:--no-e5 dense:--mode_dense}; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//_/ }
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 $flags > gpurun_out/compose/$name.log 2>&1 || { tail -20 gpurun_out/compose/$name.log; exit 1; }
  echo "$name: $(grep '\[bench\] 20 steps' gpurun_out/compose/$name.log | cut -c1-200)"
done
