#!/bin/bash
# Round 6: K2b's fp32 bound over the item's head slots only (wave-uniform skip, branch-free add) -- BM25 parity
# tests on the product, then the standalone probe kernel trace and the headline step, old vs new, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k2b; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_dropin.py \
  tests/test_gpu_multidev.py -k "bm25 or BM25 or retrieve or golden" > gpurun_out/k2b/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/k2b/tests.log; exit 1; }
tail -1 gpurun_out/k2b/tests.log
VARIANTS="variants/lib_old.so variants/lib_new.so variants/lib_newbf.so variants/lib_old.so variants/lib_new.so variants/lib_newbf.so" bash tools/k2_kprof.sh 2>&1 | grep -E "==|block_kernel|tail_kernel"
VARS="old new newbf old new newbf" bash tools/r6_ab.sh
