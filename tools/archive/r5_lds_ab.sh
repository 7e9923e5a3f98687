#!/bin/bash
# round 5: K1q LDS 160 vs 131 KiB (room for a BM25 block beside each K1q workgroup) with the deferred fallback,
# headline-only bench, alternating; then one kernel trace of the 131 KiB variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/lds; export TMPDIR=/tmp
for v in base lds131 base lds131; do
  if [ $v = base ]; then lib=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; else lib=$PWD/variants/lib_$v.so; fi
  CLASSMATE_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/lds/bench_$v.log 2>&1 || { tail -20 gpurun_out/lds/bench_$v.log; exit 1; }
  grep "steps in" gpurun_out/lds/bench_$v.log | sed "s/^/$v /" | cut -c1-330
done
CLASSMATE_HIP_LIB=$PWD/variants/lib_lds131.so timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/lds/tr -o tr --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/lds/trace.log 2>&1 || { tail -20 gpurun_out/lds/trace.log; exit 1; }
grep "steps in" gpurun_out/lds/trace.log | cut -c1-200
