#!/bin/bash
# GPU: A/B of library builds (variants/lib_<name>.so) on the same box for the 10M BM25 pruned search
# (+ identity check against the full K2 scan).  VARS="old new old new" by default.
cd "${GRAFT_REPO_ROOT:-.}"
for v in ${VARS:-old new old new}; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python tools/bm25_probe.py --paths 1,2 --reps 5 2>&1 | grep "path=2" | sed "s/^/$v /" | cut -c1-140
done
