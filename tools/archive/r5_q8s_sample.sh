#!/bin/bash
# round 5: K1q-s seed-sample fraction sweep (CM_K1QS_SAMPLE = 1/fraction of the rows in the f16 seed pass),
# 10M x 768, B = 1 and 16, k = 24 / 10
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for f in 16 32 64 128; do
  for b in 1 16; do
    CM_K1QS_SAMPLE=$f timeout -k 10 300 python -u tools/dense_probe.py --batch $b --k 24 --reps 15 2>&1 | tail -1 | sed "s/^/sample=1\/$f /"
  done
done
