#!/bin/bash
# round 5: K2a length from the postings (post_dl, K2A_PDL=1 product) vs the dl[doc] gather (variant pdl0):
# BM25 tests, bm25_probe (10M B=256) alternating, headline step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pdl; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; v0=$PWD/variants/lib_pdl0.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "bm25 or BM25" > gpurun_out/pdl/pytest.log 2>&1 || { tail -30 gpurun_out/pdl/pytest.log; exit 1; }
tail -1 gpurun_out/pdl/pytest.log
for r in 1 2; do
  for v in pdl1 pdl0; do
    L=$base; [ $v = pdl0 ] && L=$v0
    CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u tools/bm25_probe.py --paths 1,2 --reps 10 > gpurun_out/pdl/probe_$v.log 2>&1 || { tail -20 gpurun_out/pdl/probe_$v.log; exit 1; }
    grep "path=2" gpurun_out/pdl/probe_$v.log | sed "s/^/$v /" | cut -c1-170
  done
done
for v in pdl1 pdl0; do
  L=$base; [ $v = pdl0 ] && L=$v0
  CLASSMATE_HIP_LIB=$L timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/pdl/bench_$v.log 2>&1 || { tail -20 gpurun_out/pdl/bench_$v.log; exit 1; }
  grep "steps in" gpurun_out/pdl/bench_$v.log | sed "s/^/$v /" | cut -c1-330
done
