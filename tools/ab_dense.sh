#!/bin/bash
# GPU: A/B of library builds on the same box (interleaved runs): every variants/lib_*.so
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do for f in variants/lib_*.so; do
  v=$(basename $f .so)
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --path 3 --reps 7 2>&1 | grep docs= | sed "s/^/$v /" | cut -c1-105
done; done
