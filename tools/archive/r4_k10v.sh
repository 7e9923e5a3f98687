#!/bin/bash
# round 4, GPU box: K10 schedule variants (variants/lib_k10_*.so) -- accuracy tests, then GEMM + E5
# timings alternating with the product twice; then the fp32 ingest encode per-kernel profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10v; export TMPDIR=/tmp
K10_E5=1 bash tools/k10_var.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ingprof -o run --output-format csv -- python3 bench.py --mode ingest --batch 256 --seq-len 256 --steps 5 --warmup 2 --e5-dtype float32 > gpurun_out/ingprof.log 2>&1 || { tail -5 gpurun_out/ingprof.log; exit 1; }
tail -1 gpurun_out/ingprof.log | cut -c1-200
python3 tools/kstats.py gpurun_out/ingprof > gpurun_out/ingest_fp32_kernels.txt && head -25 gpurun_out/ingest_fp32_kernels.txt
