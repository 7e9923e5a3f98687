#!/bin/bash
# K10 counted waits that leave the previous tile's epilogue stores in flight (product) vs draining
# them (variants/lib_k10_noepiwait.so): GEMM + E5 accuracy tests on the product, then timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/epiw; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_scale.py -k "linear or e5 or plane or attention" -x -q --timeout 300 --timeout-method thread > gpurun_out/epiw/tests.log 2>&1 || { tail -30 gpurun_out/epiw/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/epiw/tests.log)"
for rep in 1 2; do for f in product variants/lib_k10_noepiwait.so; do
  if [ "$f" = product ]; then unset CLASSMATE_HIP_LIB; n=product; else export CLASSMATE_HIP_LIB=$PWD/$f; n=$(basename $f .so); fi
  K10_E5=1 timeout -k 10 200 python tools/k10_probe.py > gpurun_out/epiw/${n}_$rep.log 2>&1 || { tail -5 gpurun_out/epiw/${n}_$rep.log; exit 1; }
  grep -E "K10 |E5 query encode B=256 S=24 fp32 K10" gpurun_out/epiw/${n}_$rep.log | sed "s/^/$n /" | cut -c1-100
done; done
