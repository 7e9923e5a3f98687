#!/bin/bash
# GPU: split-kernel ablations (CM_DENSE_DEBUG bits) for path $PATHS at the bench shape, + PMC of the base.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/abl; export TMPDIR=/tmp
for p in ${PATHS:-3}; do
for d in ${DBG:-0 1 2 3 4 8 12 15}; do
  CM_DENSE_DEBUG=$d timeout -k 10 300 python tools/dense_probe.py --path $p --reps 3 > gpurun_out/abl/d_${p}_$d.log 2>&1 || { tail -20 gpurun_out/abl/d_${p}_$d.log; exit 1; }
  echo "path=$p dbg=$d: $(tail -1 gpurun_out/abl/d_${p}_$d.log | cut -c1-140)"
done
done
if [ "${PMC:-1}" = "1" ]; then
  bash tools/pmc.sh dense3 dense_split_kernel -- python3 tools/dense_probe.py --path 3 --reps 2 || exit 1
fi
