#!/bin/bash
# round 5: K9P (attention on the QKV planes) + the single-branch GELU -- GEMM/attention/E5 tests, the
# ingest encode (256 x 256 tokens, fp32) K9P vs K9L (CM_E5_PLANES_ATTN=0) and the headline step with the
# GELU vs the ocml-erff variant (variants/lib_k10_gelu_ocml.so), alternating; an ingest kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k9p; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; v0=$PWD/variants/lib_k10_gelu_ocml.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_engine.py -k "gemm or f16x3 or attention or e5 or E5 or planes or gelu" > gpurun_out/k9p/pytest.log 2>&1 || { tail -40 gpurun_out/k9p/pytest.log; exit 1; }
tail -1 gpurun_out/k9p/pytest.log
grep -E "planes attention|long attention S=256|K10 6144|K10 8192" gpurun_out/k9p/pytest.log | head -30
for r in 1 2; do
  for v in 1 0; do
    CM_E5_PLANES_ATTN=$v timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/k9p/ingest_$v.log 2>&1 || { tail -20 gpurun_out/k9p/ingest_$v.log; exit 1; }
    echo "planes=$v $(tail -1 gpurun_out/k9p/ingest_$v.log | cut -c1-200)"
  done
done
for r in 1 2; do
  for v in new ocml; do
    L=$base; [ $v = ocml ] && L=$v0
    CLASSMATE_HIP_LIB=$L timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/k9p/bench_$v.log 2>&1 || { tail -20 gpurun_out/k9p/bench_$v.log; exit 1; }
    echo "gelu=$v $(grep 'steps in' gpurun_out/k9p/bench_$v.log | cut -c1-200)"
    grep "ingest_fp32" gpurun_out/k9p/bench_$v.log | sed "s/^/gelu=$v /"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k9p/prof -o run --output-format csv -- python3 bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/k9p/prof.log 2>&1 || { tail -20 gpurun_out/k9p/prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/k9p/prof > gpurun_out/k9p/kernels.txt && head -12 gpurun_out/k9p/kernels.txt | cut -c1-150
