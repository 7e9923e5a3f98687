#!/bin/bash
# round 5: K2s sample size (first 1024 / 4096 / 16384 postings of the rarest walked term): BM25 tests, bm25_probe
# (10M B=256, standalone search incl. K2s) and the headline step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/scap; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so
CLASSMATE_HIP_LIB=$PWD/variants/lib_s4k.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "bm25 or BM25" > gpurun_out/scap/pytest.log 2>&1 || { tail -30 gpurun_out/scap/pytest.log; exit 1; }
tail -1 gpurun_out/scap/pytest.log
for v in base s4k s16k; do
  L=$base; [ $v != base ] && L=$PWD/variants/lib_$v.so
  CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u tools/bm25_probe.py --paths 2 --reps 10 > gpurun_out/scap/probe_$v.log 2>&1 || { tail -20 gpurun_out/scap/probe_$v.log; exit 1; }
  grep "path=2" gpurun_out/scap/probe_$v.log | sed "s/^/$v /" | cut -c1-140
done
for r in 1 2; do
  for v in base s4k; do
    L=$base; [ $v != base ] && L=$PWD/variants/lib_$v.so
    CLASSMATE_HIP_LIB=$L timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/scap/bench_$v.log 2>&1 || { tail -20 gpurun_out/scap/bench_$v.log; exit 1; }
    grep "steps in" gpurun_out/scap/bench_$v.log | sed "s/^/$v /" | cut -c1-330
  done
done
