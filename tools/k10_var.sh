#!/bin/bash
# K10 compile-time variants (variants/lib_k10_*.so, tools/build_k10_variant.sh) against the product
# library: GEMM accuracy + E5-vs-HF tests, then GEMM and fp32 E5 encode timings, twice, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10v; export TMPDIR=/tmp
for f in variants/lib_k10_*.so; do
  n=$(basename $f .so)
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread -k "linear or e5_query" > gpurun_out/k10v/test_$n.log 2>&1 || { echo "$n: tests FAILED"; tail -20 gpurun_out/k10v/test_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/k10v/test_$n.log)"
done
for rep in 1 2; do for f in product variants/lib_k10_*.so; do
  if [ "$f" = product ]; then unset CLASSMATE_HIP_LIB; n=product; else export CLASSMATE_HIP_LIB=$PWD/$f; n=$(basename $f .so); fi
  timeout -k 10 300 python -u tools/k10_probe.py > gpurun_out/k10v/probe_${n}_$rep.log 2>&1 || { tail -20 gpurun_out/k10v/probe_${n}_$rep.log; exit 1; }
  grep -E "K10|E5 query encode B=256 S=24 fp32 K10" gpurun_out/k10v/probe_${n}_$rep.log | grep -v "torch fp32 *[0-9.]* us" | sed "s/^/[$n] /"
  grep -E "^(qkv|o |up|down)" gpurun_out/k10v/probe_${n}_$rep.log | awk -v n=$n '{print "["n"] "$1" "$5" "$6}'
done; done
