#!/bin/bash
# round 5: K2a length gather behind a block-level bound (K2A_DLB=1) vs the product; bm25_probe 10M B=256 + tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/dlb; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; v=$PWD/variants/lib_dlb.so
CLASSMATE_HIP_LIB=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "bm25 or BM25" > gpurun_out/dlb/pytest.log 2>&1 || { tail -40 gpurun_out/dlb/pytest.log; exit 1; }
tail -1 gpurun_out/dlb/pytest.log
for r in 1 2; do
  for t in base dlb; do
    L=$base; [ $t = dlb ] && L=$v
    CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u tools/bm25_probe.py --paths 2 --reps 10 > gpurun_out/dlb/probe_$t.log 2>&1 || { tail -20 gpurun_out/dlb/probe_$t.log; exit 1; }
    grep "path=2" gpurun_out/dlb/probe_$t.log | sed "s/^/$t /" | cut -c1-150
  done
done
