#!/bin/bash
# GPU: K1s (B=16) and K1c (B=256) timing of variants/lib_*.so, interleaved.
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do for f in variants/lib_*.so; do for b in ${BATCHES:-16}; do
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --reps 9 --batch $b 2>&1 | grep docs= | sed "s/^/$(basename $f .so) /" | cut -c1-120
done; done; done
