#!/bin/bash
# GPU: K1c compile-time ablations (CM_DENSE_ABL) x epilogue on/off, + PMC of the base scan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/abl; export TMPDIR=/tmp
for a in 0 1 2 3; do for d in 1; do
  CM_DENSE_ABL=$a CM_DENSE_DEBUG=$d timeout -k 10 300 python tools/dense_probe.py --path 3 --reps 4 > gpurun_out/abl/a_${a}_$d.log 2>&1 || { tail -20 gpurun_out/abl/a_${a}_$d.log; exit 1; }
  echo "abl=$a dbg=$d: $(tail -1 gpurun_out/abl/a_${a}_$d.log | cut -c1-120)"
done; done
if [ "${PMC:-1}" = "1" ]; then
  CM_DENSE_DEBUG=1 bash tools/pmc.sh k1c dense_coarse_kernel -- python3 tools/dense_probe.py --path 3 --reps 2 || exit 1
fi
