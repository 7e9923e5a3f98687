#!/bin/bash
# GPU: A/B of two library builds on the same box (interleaved runs): variants/lib_old.so vs lib_new.so
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do for v in old new; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python tools/dense_probe.py --path 3 --reps 7 2>&1 | grep docs= | sed "s/^/$v /" | cut -c1-105
done; done
