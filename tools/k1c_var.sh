#!/bin/bash
# K1c compile-time variants (variants/lib_k1c*.so, tools/build_dense_variant.sh) against the product
# library: the 1M x 768 dense parity test (B = 256 / 16 / 1 vs exact fp64), then 10M x 768 B = 256
# timings, three times, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k1cv; export TMPDIR=/tmp
for f in variants/lib_k1c*.so; do
  n=$(basename $f .so)
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "dense_1m" > gpurun_out/k1cv/test_$n.log 2>&1 || { echo "$n: tests FAILED"; tail -20 gpurun_out/k1cv/test_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/k1cv/test_$n.log)"
done
for rep in 1 2 3; do for f in product variants/lib_k1c*.so; do
  if [ "$f" = product ]; then unset CLASSMATE_HIP_LIB; n=product; else export CLASSMATE_HIP_LIB=$PWD/$f; n=$(basename $f .so); fi
  timeout -k 10 300 python -u tools/dense_probe.py --reps 9 > gpurun_out/k1cv/probe_${n}_$rep.log 2>&1 || { tail -20 gpurun_out/k1cv/probe_${n}_$rep.log; exit 1; }
  grep docs= gpurun_out/k1cv/probe_${n}_$rep.log | cut -c1-200 | sed "s/^/[$n] /"
done; done
