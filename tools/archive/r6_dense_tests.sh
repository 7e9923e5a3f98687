#!/bin/bash
# Round 6: the dense parity tests (K1q / K1q-s / prefix plane / 10M sample / 1M dense / drop-in) on the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/dt; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_f16_prefix.py \
  tests/test_gpu_engine.py tests/test_gpu_dropin.py "tests/test_gpu_scale.py::test_hybrid_10m_sample" "tests/test_gpu_scale.py::test_dense_1m_x_768" \
  > gpurun_out/dt/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/dt/tests.log; exit 1; }
tail -1 gpurun_out/dt/tests.log
