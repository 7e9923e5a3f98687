#!/bin/bash
# GPU: A/B of two library builds on the same box for the 10M BM25 pruned search (+ identity check)
cd "${GRAFT_REPO_ROOT:-.}"
for v in old new old new; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python tools/bm25_probe.py --paths 1,2 --reps 5 2>&1 | grep "path=2" | sed "s/^/$v /" | cut -c1-140
done
