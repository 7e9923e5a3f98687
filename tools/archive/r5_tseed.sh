#!/bin/bash
# round 5: K2s seeded threshold for the BM25 tail pass -- BM25 tests (product and the K2A_PREB=1 variant), then
# tools/bm25_probe.py (10M, B=256; full vs pruned, identical results) and the headline step, seed on/off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/tseed; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; pb=$PWD/variants/lib_preb1.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "bm25 or BM25" > gpurun_out/tseed/pytest_base.log 2>&1 || { tail -40 gpurun_out/tseed/pytest_base.log; exit 1; }
tail -1 gpurun_out/tseed/pytest_base.log
CLASSMATE_HIP_LIB=$pb timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py -k "bm25 or BM25" > gpurun_out/tseed/pytest_preb1.log 2>&1 || { tail -40 gpurun_out/tseed/pytest_preb1.log; exit 1; }
tail -1 gpurun_out/tseed/pytest_preb1.log
for lib in base preb1; do
  L=$base; [ $lib = preb1 ] && L=$pb
  for sd in 1 0; do
    CM_BM25_TSEED=$sd CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u tools/bm25_probe.py --paths 1,2 --reps 10 > gpurun_out/tseed/probe_${lib}_$sd.log 2>&1 || { tail -20 gpurun_out/tseed/probe_${lib}_$sd.log; exit 1; }
    grep "path=2" gpurun_out/tseed/probe_${lib}_$sd.log | sed "s/^/$lib seed=$sd /" | cut -c1-260
  done
done
for v in base_1 base_0 preb1_1; do
  lib=${v%_*}; sd=${v#*_}; L=$base; [ $lib = preb1 ] && L=$pb
  CM_BM25_TSEED=$sd CLASSMATE_HIP_LIB=$L timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/tseed/bench_$v.log 2>&1 || { tail -20 gpurun_out/tseed/bench_$v.log; exit 1; }
  grep "steps in" gpurun_out/tseed/bench_$v.log | sed "s/^/$v /" | cut -c1-400
done
