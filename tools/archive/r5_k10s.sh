#!/bin/bash
# round 5: K10s (skinny M <= 32 GEMM) -- GEMM tests, then batch-1 / batch-8 encode latency: tiled kernel
# (CM_K10_SKINNY=0) vs skinny at depth 8 (product) / 12 / 4, alternating; then a kernel trace of the product
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10s; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/k10s/pytest.log 2>&1 || { tail -30 gpurun_out/k10s/pytest.log; exit 1; }
tail -1 gpurun_out/k10s/pytest.log
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so
for r in 1 2; do
  for v in tiled d8 d12 d4; do
    lib=$base; env=""
    [ $v = tiled ] && env="CM_K10_SKINNY=0"
    [ $v = d12 ] && lib=$PWD/variants/lib_k10_d12.so
    [ $v = d4 ] && lib=$PWD/variants/lib_k10_d4.so
    env $env CLASSMATE_HIP_LIB=$lib timeout -k 10 200 python -u tools/e5_b1_probe.py > gpurun_out/k10s/probe_$v.log 2>&1 || { tail -20 gpurun_out/k10s/probe_$v.log; exit 1; }
    grep "E5 encode" gpurun_out/k10s/probe_$v.log | sed "s/^/$v /"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k10s/tr -o tr --output-format csv -- python3 -u tools/e5_b1_probe.py > gpurun_out/k10s/trace.log 2>&1 || { tail -20 gpurun_out/k10s/trace.log; exit 1; }
grep "E5 encode" gpurun_out/k10s/trace.log
