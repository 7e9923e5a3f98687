#!/bin/bash
# Round 6: K1q epilogue hoisted into the last chunk's MFMA gaps -- dense parity tests on the product,
# then standalone scans (tools/dense_probe.py, kind 5, B = 256) and the headline step, old vs new, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k1q; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_f16_prefix.py \
  "tests/test_gpu_scale.py::test_hybrid_10m_sample" "tests/test_gpu_scale.py::test_dense_1m_x_768" > gpurun_out/k1q/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/k1q/tests.log; exit 1; }
tail -2 gpurun_out/k1q/tests.log
for rep in 1 2; do for v in old new; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python tools/dense_probe.py --path 5 --reps 7 > gpurun_out/k1q/probe_$v$rep.log 2>&1 \
    || { echo "probe $v failed"; tail -20 gpurun_out/k1q/probe_$v$rep.log; exit 1; }
  grep "docs=" gpurun_out/k1q/probe_$v$rep.log | sed "s/^/$v /" | cut -c1-160
done; done
VARS="old new old new" bash tools/r6_ab.sh
