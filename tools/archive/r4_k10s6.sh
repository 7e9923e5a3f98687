#!/bin/bash
# GPU: product with the 6-stage 64 x 32 K10 tile -- GEMM + drop-in tests, batch-1 E5 latency
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10s6; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_dropin.py -x -q --timeout 240 --timeout-method thread > gpurun_out/k10s6/t.log 2>&1 || { tail -30 gpurun_out/k10s6/t.log; exit 1; }
tail -1 gpurun_out/k10s6/t.log
timeout -k 10 200 python -u tools/e5_b1_probe.py 2>&1 | grep "E5 encode"
