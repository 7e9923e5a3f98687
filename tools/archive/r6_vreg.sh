#!/bin/bash
# Round 6 (late): K1Q_VREG variant -- dense parity tests on it, standalone scan probe, then the step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
CLASSMATE_HIP_LIB=$PWD/variants/lib_vreg.so timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
  tests/test_gpu_q8.py > gpurun_out/vreg_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/vreg_tests.log | tail -8
[ $rc -eq 0 ] || { tail -40 gpurun_out/vreg_tests.log; exit 1; }
for v in base vreg base vreg; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python tools/dense_probe.py --path 5 --reps 7 > gpurun_out/vreg_probe.log 2>&1 || { tail -20 gpurun_out/vreg_probe.log; exit 1; }
  grep docs= gpurun_out/vreg_probe.log | sed "s/^/$v /" | cut -c1-140
done
VARS=${VARS:-"base vreg base vreg"} bash tools/r6_ab.sh
