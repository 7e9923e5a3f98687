#!/bin/bash
# Round 6: (1) seed-sample env A/B; (2) K2a pre-bound on the 16-doc sub-block maxima (variants/lib_p3.so, -DK2A_PREB=3):
# BM25 parity tests on it, the standalone probe's kernel trace (base / p1 / p3), the headline step base vs p3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/p3; export TMPDIR=/tmp
ENVS="base s32=CM_K1Q_SAMPLE=32" REPS=2 bash tools/r6_env_ab.sh || exit 1
CLASSMATE_HIP_LIB=$PWD/variants/lib_p3.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_engine.py tests/test_gpu_dropin.py -k "bm25 or BM25 or retrieve or golden" > gpurun_out/p3/tests.log 2>&1 \
  || { echo "p3 tests failed"; tail -30 gpurun_out/p3/tests.log; exit 1; }
tail -1 gpurun_out/p3/tests.log
VARIANTS="variants/lib_base.so variants/lib_p1.so variants/lib_p3.so" bash tools/k2_kprof.sh 2>&1 | grep -E "==|block_kernel|tail_kernel"
VARS="base p3 base p3" bash tools/r6_ab.sh
