#!/bin/bash
# GPU: K1c paired (default) vs whole-pass form at the bench shape, interleaved.
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do for p in 1 0; do
  CM_K1C_PAIRED=$p timeout -k 10 300 python tools/dense_probe.py --reps 9 2>&1 | grep docs= | sed "s/^/paired=$p /" | cut -c1-150
done; done
