#!/bin/bash
# Round 6: same-box A/B of library variants (variants/lib_<name>.so) in the headline step (no side legs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARS:-base u3 base u3}; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --dense-legs 0 \
    --e5-other-leg 0 --ingest-leg 0 --cpu-baseline 0 --out gpurun_out/ab_$v.json > gpurun_out/ab_$v.log 2>&1 \
    || { echo "$v failed"; tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "$v $(grep 'steps in' gpurun_out/ab_$v.log | cut -c1-330)"
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_$v.json'));print('  $v breakdown', {k:round(x,3) for k,x in d['breakdown_ms'].items() if x})"
done
