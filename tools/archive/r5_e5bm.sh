#!/bin/bash
# round 5: BM25 beside the E5 encode with K10 sized for co-residency (96 x 192 tile everywhere, 3-stage
# ring: <= 120 KiB LDS per workgroup leaves a BM25 block per CU) vs the product schedule, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e5bm; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; s3=$PWD/variants/lib_k10_s3.so
run() {  # tag lib env... -- bench args
  local tag=$1 lib=$2; shift 2
  env CLASSMATE_HIP_LIB=$lib "$@" > gpurun_out/e5bm/bench_$tag.log 2>&1 || { tail -20 gpurun_out/e5bm/bench_$tag.log; exit 1; }
  grep "steps in" gpurun_out/e5bm/bench_$tag.log | sed "s/^/$tag /" | cut -c1-330
}
B="timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0"
for r in 1 2; do
  run product $base $B
  run s3_after $s3 CM_K10_TILE=6x12 $B
  run s3_with_e5 $s3 CM_K10_TILE=6x12 $B --bm25-with-e5
  run base_with_e5 $base $B --bm25-with-e5
done
