#!/bin/bash
# round 5: K2a range-level pre-bound (K2A_PREB=2: no per-candidate load before the bound) with the seeded T,
# 5 waves/SIMD (15 spilled VGPRs) and 4 (none), vs the product (gathers first); bm25_probe at 10M B=256 + tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/preb2; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so
for v in preb2 preb2w4; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "bm25 or BM25" > gpurun_out/preb2/pytest_$v.log 2>&1 || { tail -40 gpurun_out/preb2/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/preb2/pytest_$v.log | sed "s/^/$v /"
done
for r in 1 2; do
  for v in base preb2 preb2w4; do
    L=$base; [ $v != base ] && L=$PWD/variants/lib_$v.so
    CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u tools/bm25_probe.py --paths 2 --reps 10 > gpurun_out/preb2/probe_$v.log 2>&1 || { tail -20 gpurun_out/preb2/probe_$v.log; exit 1; }
    grep "path=2" gpurun_out/preb2/probe_$v.log | sed "s/^/$v /" | cut -c1-200
  done
done
