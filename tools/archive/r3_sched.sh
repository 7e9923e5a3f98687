#!/bin/bash
# step scheduling A/B (BM25 beside the E5 encode / beside the dense scan / serial), then the N=2
# rehearsal with the recall diagnostics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/sched; export TMPDIR=/tmp
for v in "default:" "serial:--serial" "after_e5:--bm25-after-e5"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --dense-legs 0 --e5-other-leg 0 --cpu-baseline 0 $f > gpurun_out/sched/$n.log 2>&1 || { tail -20 gpurun_out/sched/$n.log; exit 1; }
  echo "$n: $(grep '\[bench\] 20 steps' gpurun_out/sched/$n.log | cut -c1-330)"
done
DOCS=1000000 bash tools/mgpu_rehearsal.sh > gpurun_out/sched/mgpu.txt 2>&1 || { tail -20 gpurun_out/sched/mgpu.txt; exit 1; }
grep -E "recall|mismatch|mmr q" gpurun_out/mgpu/rehearsal.log | cut -c1-700
