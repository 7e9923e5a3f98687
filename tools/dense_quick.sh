#!/bin/bash
# GPU: dense parity tests + the 20-step bench (dense re-rank / glue changes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "dense or vector or hybrid or retriev or golden or parallel or filter" > gpurun_out/dense_tests.log 2>&1 || { tail -30 gpurun_out/dense_tests.log; exit 1; }
tail -1 gpurun_out/dense_tests.log
VARIANTS="default:" bash tools/compose_probe.sh
