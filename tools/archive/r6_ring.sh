#!/bin/bash
# Round 6: K1q ring depth of the full-LDS form (variants/lib_r<N>.so, -DK1Q_RING_FULL=N) -- standalone scans, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ring; export TMPDIR=/tmp
if [ -n "$TESTLIB" ]; then
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$TESTLIB.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_q8.py > gpurun_out/ring/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ring/tests.log; exit 1; }
  tail -1 gpurun_out/ring/tests.log
fi
for rep in 1 2; do for v in ${VARS:-base r14 r16}; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python tools/dense_probe.py --path 5 --reps 7 > gpurun_out/ring/probe_$v$rep.log 2>&1 \
    || { echo "probe $v failed"; tail -20 gpurun_out/ring/probe_$v$rep.log; exit 1; }
  grep "docs=" gpurun_out/ring/probe_$v$rep.log | sed "s/^/$v /" | cut -c1-160
done; done
