#!/bin/bash
# round 5: K9P at 8 waves per workgroup (two per CU, XCD-paired query blocks) vs 16 (variants/lib_k9p16.so):
# attention/E5 tests, ingest encode alternating, ingest kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k9p3; export TMPDIR=/tmp
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; v16=$PWD/variants/lib_k9p16.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm.py -k "planes or attention or e5 or qkv" > gpurun_out/k9p3/pytest.log 2>&1 || { tail -40 gpurun_out/k9p3/pytest.log; exit 1; }
tail -1 gpurun_out/k9p3/pytest.log
for r in 1 2; do
  for v in w8 w16; do
    L=$base; [ $v = w16 ] && L=$v16
    CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 10 --warmup 3 > gpurun_out/k9p3/ingest_$v.log 2>&1 || { tail -20 gpurun_out/k9p3/ingest_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/k9p3/ingest_$v.log | cut -c1-200)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k9p3/prof -o run --output-format csv -- python3 bench.py --mode ingest --e5-dtype float32 --seq-len 256 --steps 5 --warmup 2 > gpurun_out/k9p3/prof.log 2>&1 || { tail -20 gpurun_out/k9p3/prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/k9p3/prof > gpurun_out/k9p3/kernels.txt && head -8 gpurun_out/k9p3/kernels.txt | cut -c1-150
