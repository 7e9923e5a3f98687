#!/bin/bash
# GPU: K10 64 x 32 tile for M <= 32 -- GEMM accuracy + tile-independence tests, drop-in tests, batch-1 E5 latency
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10s; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 240 --timeout-method thread > gpurun_out/k10s/gemm.log 2>&1 || { tail -30 gpurun_out/k10s/gemm.log; exit 1; }
tail -1 gpurun_out/k10s/gemm.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 240 --timeout-method thread > gpurun_out/k10s/dropin.log 2>&1 || { tail -30 gpurun_out/k10s/dropin.log; exit 1; }
tail -1 gpurun_out/k10s/dropin.log
timeout -k 10 300 python -u tools/e5_b1_probe.py 2>&1 | tee gpurun_out/k10s/probe.log | grep "E5 encode"
