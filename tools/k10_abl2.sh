#!/bin/bash
# K10 ablation ladder (variants/lib_k10_*.so, results wrong by design) beside the product, per GEMM
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10abl; export TMPDIR=/tmp
for rep in 1 2; do for f in product variants/lib_k10_*.so; do
  if [ "$f" = product ]; then unset CLASSMATE_HIP_LIB; n=product; else export CLASSMATE_HIP_LIB=$PWD/$f; n=$(basename $f .so); fi
  K10_E5=0 timeout -k 10 120 python tools/k10_probe.py > gpurun_out/k10abl/${n}_$rep.log 2>&1 || { tail -5 gpurun_out/k10abl/${n}_$rep.log; exit 1; }
  grep -E "K10 " gpurun_out/k10abl/${n}_$rep.log | awk -v n=$n '{print n, $1, $6, $7}'
done; done
